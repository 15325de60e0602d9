#!/bin/bash
# r5: confirm the new defaults (keepWarmMs 10 + idleWakeMs 1) against keepWarmMs 1: bench
# alternated four times per setting (warm p50/p99.9, cold = calls 1 ms apart), then the idle
# probe over 1 ms .. 1 s gaps with the defaults, then the GPU tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$PWD/gpurun_out/r5"
mkdir -p "$OUT"
: > "$OUT/ab_defaults.jsonl"
for i in 1 2 3 4; do
  for arm in default kw1; do
    if [ $arm = kw1 ]; then cfg='{"grpc": {"keepWarmMs": 1, "idleWakeMs": 0}}'; else cfg=''; fi
    echo "=== bench $arm #$i ($(date +%T))"
    timeout -k 10 300 python bench.py ${cfg:+--daemon-config "$cfg"} > "$OUT/bench_def_$arm.log" 2>&1 || exit $?
    tail -1 "$OUT/bench_def_$arm.log" | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print(json.dumps({'arm': '$arm', 'round': $i, 'p50': d['value'], 'p99': d['allocate_p99_us'], 'p999': d['allocate_p999_us'],
                  'cold': d['allocate_cold_p50_us'], 'cold_floor': d['uds_roundtrip_floor_cold_p50_us'],
                  'admission': d['allocate_admission_p50_us'], 'floor_batched': d['uds_roundtrip_floor_batched_us'],
                  'other': d['allocate_tail']['other']}))" | tee -a "$OUT/ab_defaults.jsonl"
    if [ $arm = default ] && [ $i = 1 ]; then cp "$OUT/bench_def_default.log" "$OUT/bench_def_default_1.log"; fi
  done
done
echo "=== idle gaps, defaults ($(date +%T))"
timeout -k 10 700 python -u scripts/idle_probe.py --gaps 0.001,0.01,0.1,1 --calls 60 \
  --out "$OUT/idle_probe_gaps_defaults.json" > "$OUT/idle_gaps_defaults.log" 2>&1 || exit $?
grep attribution "$OUT/idle_gaps_defaults.log" | cut -c1-1500
echo "=== pytest gpu ($(date +%T))"
timeout -k 10 420 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || exit $?
tail -2 "$OUT/gpu_tests.log"
echo "=== done"
