#!/bin/bash
# r6: the current tree on one lease - GPU tests, smoke, the driver's bench command (with
# the canary) twice, the reset-query probe, the idle cost, and a rocprofv3 kernel trace
# of the smoke run's canary kernels.  Outputs under gpurun_out/r6/<tag>_*.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-final}
OUT="$PWD/gpurun_out/r6"
mkdir -p "$OUT"
echo "=== pytest gpu ($(date +%T))"
timeout -k 10 420 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/${tag}_gpu_tests.log" 2>&1 || exit $?
tail -1 "$OUT/${tag}_gpu_tests.log"
echo "=== smoke ($(date +%T))"
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${tag}_smoke.log" 2>&1 || exit $?
tail -1 "$OUT/${tag}_smoke.log"
for i in 1 2; do
  echo "=== bench #$i ($(date +%T))"
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/${tag}_bench_$i.json" 2> "$OUT/${tag}_bench_$i.err" || exit $?
  python3 -c "
import json
d = json.loads(open('$OUT/${tag}_bench_$i.json').read().strip().splitlines()[-1])
print(json.dumps({'p50': d['value'], 'floor_spin': d['uds_roundtrip_floor_spin_p50_us'], 'paired': d['allocate_vs_spin_floor_paired'],
                  'p999': d['allocate_p999_us'], 'rps': d['scrape_rps']}))"
done
echo "=== reset query probe ($(date +%T))"
timeout -k 10 120 python scripts/reset_query_probe.py --out "$OUT/${tag}_reset_query_probe.json" > /dev/null 2>&1 || exit $?
echo "=== idle cost ($(date +%T))"
timeout -k 10 240 python scripts/idle_wakeups.py --settle 130 --out "$OUT/${tag}_idle_wakeups.json" > "$OUT/${tag}_idle_wakeups.log" 2>&1 || exit $?
tail -3 "$OUT/${tag}_idle_wakeups.log" | head -2
echo "=== rocprofv3 smoke ($(date +%T))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${tag}_prof" -o smoke -- python3 -c "import sys; sys.path.insert(0, '$GRAFT_REPO_ROOT'); import __graft_entry__ as g; g.smoke()" > "$OUT/${tag}_prof.log" 2>&1 || exit $?
echo "=== done ($(date +%T))"
