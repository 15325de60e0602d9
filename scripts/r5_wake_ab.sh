#!/bin/bash
# r5: what keeps the first call after a long idle fast - running the request path every
# idle millisecond (keepWarmMs 1) or only waking every millisecond (idleWakeMs 1, the path
# every 10 ms)?  The 1 s-idle probe with one daemon per setting, calls interleaved, and
# bench.py per setting (its cold case: calls 1 ms apart).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$PWD/gpurun_out/r5"
mkdir -p "$OUT"
ARMS='{"kw1": {"grpc": {"keepWarmMs": 1, "idleWakeMs": 0}}, "kw10wake1": {"grpc": {"keepWarmMs": 10, "idleWakeMs": 1}}, "kw10": {"grpc": {"keepWarmMs": 10, "idleWakeMs": 0}}}'
: > "$OUT/ab_wake_bench.jsonl"
for arm in kw1 kw10wake1 kw10; do
  cfg=$(python3 -c "import json,sys; print(json.dumps(json.loads(sys.argv[1])[sys.argv[2]]))" "$ARMS" "$arm")
  echo "=== bench $arm ($(date +%T))"
  timeout -k 10 300 python bench.py --daemon-config "$cfg" > "$OUT/bench_$arm.log" 2>&1 || exit $?
  tail -1 "$OUT/bench_$arm.log" | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print(json.dumps({'arm': '$arm', 'p50': d['value'], 'p999': d['allocate_p999_us'], 'cold': d['allocate_cold_p50_us'],
                  'cold_floor': d['uds_roundtrip_floor_cold_p50_us'], 'admission': d['allocate_admission_p50_us']}))" | tee -a "$OUT/ab_wake_bench.jsonl"
done
echo "=== idle A/B ($(date +%T))"
timeout -k 10 600 python -u scripts/idle_probe.py --gaps 1 --calls ${IDLE_CALLS:-75} --rpcs allocate \
  --ab-overrides "$ARMS" --out "$OUT/idle_ab_wake.json" > "$OUT/idle_ab_wake.log" 2>&1 || exit $?
python3 -c "
import json; d = json.load(open('$OUT/idle_ab_wake.json'))
for r in d['rows']:
  for k, v in r.items():
    if isinstance(v, dict): print(k, {x: v.get(x) for x in ('p50_us', 'minus_floor_median_us', 'minus_floor_ci95_us', 'median_us', 'ci95_us', 'segments_p50_us')})
print(d['daemon_cpu_percent'])"
echo "=== done"
