"""HBM access-shape sweep at the canary's sizes (1 GiB bench, 2 GiB rocprof) and 4 GiB."""
import json
import sys

from k8s_gpu_device_plugin_amd.ops import canary

rows = []
for nbytes in (1 << 30, 4 << 30):
    for r in canary.hbm_sweep(0, nbytes, variants=(4, 5, 6, 8, 9, 10, 11, 12), blocks_per_cu=(4, 8, 16, 32), reps=10):
        r["bytes"] = nbytes
        rows.append(r)
        print(json.dumps(r), flush=True)
json.dump(rows, open(sys.argv[1], "w"), indent=1)
