import json, sys
from k8s_gpu_device_plugin_amd.ops import canary
bad = 0
for kk in sys.argv[1:]:
    for shp in [(256, 256, 64), (256, 256, 192), (1024, 2048, 640), (2048, 1024, 4096), (4096, 4096, 4096)]:
        r = canary.gemm_rate(0, *shp, iters=2, kernel=kk)
        bad += r["errors"] != 0
        if r["errors"]: print("ERR", kk, shp, r)
print("exactness screen:", "ok" if not bad else "FAILED")
sys.exit(1 if bad else 0)
