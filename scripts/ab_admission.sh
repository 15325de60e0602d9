#!/bin/bash
# A/B of grpc.admissionPollUs (0 vs the 1000 us default), alternating runs of bench.py in
# one gpurun call; prints the Allocate latencies of each run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$PWD/gpurun_out"
mkdir -p "$OUT"
for i in 1 2; do
  for a in 0 1000; do
    timeout -k 10 240 python bench.py --no-canary --steps 10 --warmup 2 --admission-poll-us $a > "$OUT/ab_adm_${a}_$i.log" 2>&1 || exit $?
    grep '^{' "$OUT/ab_adm_${a}_$i.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('admissionPollUs=$a', {k: d[k] for k in ('allocate_p50_us', 'allocate_cold_p50_us', 'allocate_admission_p50_us', 'uds_roundtrip_floor_p50_us', 'uds_roundtrip_floor_spin_p50_us')})"
  done
done
