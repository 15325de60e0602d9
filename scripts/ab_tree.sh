cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in 1 2 3 4; do
  for t in . ab_old; do
    (cd $t && timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-canary 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['value'], d['uds_roundtrip_floor_spin_p50_us'], d['uds_roundtrip_floor_p50_us'], d['allocate_cold_p50_us'], d['scrape_rps'])") >> gpurun_out/ab.txt || exit 1
  done
done
