#!/bin/bash
# r5: the call-trace ring is written through once at set-up (a page's first write faulted
# inside every 73rd traced request).  bench.py four times (tail causes, p99), then the idle
# probe's daemon fault counters at 1 ms gaps, then the GPU tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$PWD/gpurun_out/r5"
mkdir -p "$OUT"
: > "$OUT/prefault_bench.jsonl"
for i in 1 2 3 4; do
  echo "=== bench #$i ($(date +%T))"
  timeout -k 10 300 python bench.py > "$OUT/bench_prefault_$i.log" 2>&1 || exit $?
  tail -1 "$OUT/bench_prefault_$i.log" | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); t = d['allocate_tail']
print(json.dumps({'round': $i, 'p50': d['value'], 'p99': d['allocate_p99_us'], 'p999': d['allocate_p999_us'], 'max': d['allocate_max_us'],
                  'by_cause': t['by_cause'], 'excess': t.get('cause_mean_excess_us'), 'other': t['other'],
                  'floor_batched': d['uds_roundtrip_floor_batched_us'], 'cold': d['allocate_cold_p50_us'],
                  'cold_floor': d['uds_roundtrip_floor_cold_p50_us'], 'scrape_rps': d['scrape_rps']}))" | tee -a "$OUT/prefault_bench.jsonl"
done
echo "=== idle probe 1 ms ($(date +%T))"
timeout -k 10 300 python -u scripts/idle_probe.py --gaps 0.001 --calls 300 --out "$OUT/idle_probe_prefault.json" > "$OUT/idle_prefault.log" 2>&1 || exit $?
python3 -c "
import json; d = json.load(open('$OUT/idle_probe_prefault.json'))
for r in d['rows']: print(r['gap_s'], r['allocate']['p50_us'], r['allocate']['per_call'])"
echo "=== pytest gpu ($(date +%T))"
timeout -k 10 420 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || exit $?
tail -2 "$OUT/gpu_tests.log"
echo "=== done"
