#!/bin/bash
# r5: the current tree - GPU tests, smoke, bench three times.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$PWD/gpurun_out/r5"
mkdir -p "$OUT"
echo "=== pytest gpu ($(date +%T))"
timeout -k 10 420 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || exit $?
tail -1 "$OUT/gpu_tests.log"
echo "=== smoke ($(date +%T))"
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
tail -1 "$OUT/smoke.log"
: > "$OUT/final_bench.jsonl"
for i in 1 2 3; do
  echo "=== bench #$i ($(date +%T))"
  timeout -k 10 300 python bench.py > "$OUT/bench_final_$i.log" 2>&1 || exit $?
  tail -1 "$OUT/bench_final_$i.log" | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print(json.dumps({'round': $i, 'p50': d['value'], 'p99': d['allocate_p99_us'], 'p999': d['allocate_p999_us'],
                  'floor_spin': d['uds_roundtrip_floor_spin_p50_us'], 'floor_batched': d['uds_roundtrip_floor_batched_us'],
                  'cold': d['allocate_cold_p50_us'], 'cold_floor': d['uds_roundtrip_floor_cold_p50_us'],
                  'server_mean': d['allocate_server_mean_us'], 'alloc8': d['preferred_allocator_8gpu_size4_p50_us'],
                  'scrape_rps': d['scrape_rps'], 'scrape_p50': d['scrape_p50_us'], 'scrape_server_mean': d['scrape_server_mean_us'],
                  'by_cause': d['allocate_tail']['by_cause'], 'other': d['allocate_tail']['other']}))" | tee -a "$OUT/final_bench.jsonl"
done
echo "=== done"
