# A/B of bench.py between this tree (.) and ./ab_old, alternating on one box; the order
# within a pair flips every pair.  PAIRS (default 4) pairs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in $(seq 1 ${PAIRS:-4}); do
  if [ $((i % 2)) -eq 1 ]; then order=". ab_old"; else order="ab_old ."; fi
  for t in $order; do
    (cd $t && timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-canary 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['value'], d['allocate_p99_us'], d['uds_roundtrip_floor_spin_p50_us'], d['allocate_cold_p50_us'], d['allocate_admission_p50_us'], d['scrape_rps'])") >> gpurun_out/ab.txt || exit 1
  done
done
