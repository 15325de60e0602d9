cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in 1 2; do
  for t in . ab_old; do
    extra=""; [ "$t" = "." ] && extra="--backend fixture"
    (cd $t && HIP_VISIBLE_DEVICES=-1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
      --master-addr 127.0.0.1 --master-port $((29800 + i)) bench.py --gpus 4 --steps 10 --warmup 2 $extra 2>/dev/null \
      | grep '^{' | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['value'], d['allocate_p99_us'], d['scrape_rps'], d['scrape_p50_us'], d['metrics_bytes'], d['preferred_p50_us'])") >> gpurun_out/ab_ranks.txt || exit 1
  done
done
