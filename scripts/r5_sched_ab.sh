#!/bin/bash
# r5: do the daemon's own background threads (1 Hz telemetry pass, 25 ms watchdog, lanes)
# preempt the gRPC worker mid-request?  bench.py with backgroundSched batch (SCHED_BATCH:
# a waking batch thread never preempts) vs normal, alternated three times; then the
# keep-warm / idle-wake A/B (scripts/r5_wake_ab.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$PWD/gpurun_out/r5"
mkdir -p "$OUT"
: > "$OUT/ab_sched.jsonl"
for i in 1 2 3; do
  for s in batch normal; do
    echo "=== bench backgroundSched=$s #$i ($(date +%T))"
    timeout -k 10 300 python bench.py --daemon-config "{\"backgroundSched\": \"$s\"}" > "$OUT/bench_sched_$s.log" 2>&1 || exit $?
    tail -1 "$OUT/bench_sched_$s.log" | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); t = d['allocate_tail']
print(json.dumps({'sched': '$s', 'round': $i, 'p50': d['value'], 'p99': d['allocate_p99_us'], 'p999': d['allocate_p999_us'],
                  'max': d['allocate_max_us'], 'by_cause': t['by_cause'], 'excess': t.get('cause_mean_excess_us'),
                  'slowest': [(s['us'], s['cause']) for s in t['slowest'][:5]], 'floor_batched': d['uds_roundtrip_floor_batched_us'],
                  'cold': d['allocate_cold_p50_us'], 'cold_floor': d['uds_roundtrip_floor_cold_p50_us']}))" | tee -a "$OUT/ab_sched.jsonl"
  done
done
bash scripts/r5_wake_ab.sh
