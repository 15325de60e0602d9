#!/bin/bash
# Repeated bench.py runs in one gpurun call (box-variance check), then a 4-rank rehearsal
# of the multi-rank path with the GPU hidden from the ranks (gloo; the daemon still sees the
# real GPU through amdsmi).  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$PWD/gpurun_out"
mkdir -p "$OUT"
for i in ${REPS:-1 2 3}; do
  timeout -k 10 240 python bench.py --no-canary --steps 20 --warmup 3 > "$OUT/rep_$i.log" 2>&1 || exit $?
  grep '^{' "$OUT/rep_$i.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rep', $i, {k: d[k] for k in ('allocate_p50_us', 'allocate_p99_us', 'uds_roundtrip_floor_spin_p50_us', 'scrape_rps', 'scrape_p50_us', 'tcp_scrape_floor_p50_us')})"
done
if [ -n "${RANKS:-}" ]; then
  HIP_VISIBLE_DEVICES=-1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$RANKS" \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus "$RANKS" --no-canary --steps 10 --warmup 2 \
    > "$OUT/ranks_$RANKS.log" 2>&1 || exit $?
  grep '^{' "$OUT/ranks_$RANKS.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ranks', $RANKS, {k: d[k] for k in ('allocate_p50_us', 'allocate_p99_us', 'scrape_rps', 'scrape_p50_us', 'n_gpus')})"
fi
