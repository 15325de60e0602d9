#!/bin/bash
# r5: does the 1 Hz telemetry pass (amdsmi calls on the GPU lanes, exposition render)
# preempt the gRPC worker mid-request?  bench.py with telemetry every 1 s vs every 100 s,
# alternated; then the GPU tests on this tree.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$PWD/gpurun_out/r5"
mkdir -p "$OUT"
: > "$OUT/ab_telemetry.jsonl"
for i in 1 2 3; do
  for ms in 1000 100000; do
    echo "=== bench telemetry=${ms}ms #$i ($(date +%T))"
    timeout -k 10 300 python bench.py --daemon-config "{\"telemetry\": {\"intervalMs\": $ms}}" > "$OUT/bench_tel_$ms.log" 2>&1 || exit $?
    tail -1 "$OUT/bench_tel_$ms.log" | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); t = d['allocate_tail']
print(json.dumps({'telemetry_ms': $ms, 'round': $i, 'p50': d['value'], 'p99': d['allocate_p99_us'], 'p999': d['allocate_p999_us'],
                  'max': d['allocate_max_us'], 'by_cause': t['by_cause'], 'excess': t.get('cause_mean_excess_us'),
                  'slowest': [(s['us'], s['cause']) for s in t['slowest'][:5]], 'floor_batched': d['uds_roundtrip_floor_batched_us']}))" | tee -a "$OUT/ab_telemetry.jsonl"
  done
done
echo "=== pytest gpu ($(date +%T))"
timeout -k 10 420 python -u -m pytest tests -x -v -m gpu -s -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || exit $?
tail -2 "$OUT/gpu_tests.log"
grep -E "latch|firmware" "$OUT/gpu_tests.log" | head -5
echo "=== done"
