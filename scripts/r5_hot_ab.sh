#!/bin/bash
# r5: hot-connection recv polling (grpc.hotRecvPoll) on and off, alternated on one box,
# then the GPU tests and smoke on the same tree.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$PWD/gpurun_out/r5"
mkdir -p "$OUT"
: > "$OUT/ab_hot_recv.jsonl"
for i in 1 2 3 4; do
  for v in false true; do
    echo "=== bench hot=$v #$i ($(date +%T))"
    timeout -k 10 300 python bench.py --daemon-config "{\"grpc\": {\"hotRecvPoll\": $v}}" > "$OUT/bench_hot_$v.log" 2>&1 || exit $?
    tail -1 "$OUT/bench_hot_$v.log" | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); t = d['allocate_tail']
r = {'hot': '$v', 'round': $i, 'p50': d['value'], 'p99': d['allocate_p99_us'], 'p999': d['allocate_p999_us'],
     'floor_spin_p50': d['uds_roundtrip_floor_spin_p50_us'], 'floor_batched': d['uds_roundtrip_floor_batched_us'],
     'segments': t.get('segment_p50_us'), 'split': t.get('server_split_p50_us'), 'scrape_rps': d['scrape_rps'],
     'server_mean': d['allocate_server_mean_us']}
print(json.dumps(r))" | tee -a "$OUT/ab_hot_recv.jsonl"
  done
done
echo "=== pytest gpu ($(date +%T))"
timeout -k 10 420 python -u -m pytest tests -x -v -m gpu -s -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || exit $?
tail -2 "$OUT/gpu_tests.log"
echo "=== smoke ($(date +%T))"
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
tail -1 "$OUT/smoke.log" | cut -c1-300
echo "=== done"
