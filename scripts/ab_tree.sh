# A/B(/C) of bench.py between trees on one box, interleaved: TREES (default ". ab_old")
# are run in a rotating order, PAIRS (default 4) rounds.  Each line: tree, Allocate p50,
# p99, polling-server floor p50, cold p50, admission p50, /metrics RPS (2 connections),
# /metrics p50, /metrics body bytes, loopback-TCP floor of that body.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
read -r -a trees <<< "${TREES:-. ab_old}"
out="gpurun_out/${AB_OUT:-ab.txt}"
for i in $(seq 1 ${PAIRS:-4}); do
  k=${#trees[@]}
  for j in $(seq 0 $((k - 1))); do
    t=${trees[$(( (i + j) % k ))]}
    (cd "$t" && timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-canary 2>/dev/null | tail -1 | python -c "
import json, sys
d = json.loads(sys.stdin.read())
print('$t', d['value'], d['allocate_p99_us'], d['uds_roundtrip_floor_spin_p50_us'], d['allocate_cold_p50_us'],
      d['allocate_admission_p50_us'], d['scrape_rps'], d['scrape_p50_us'], d['metrics_bytes'], d.get('tcp_scrape_floor_p50_us'))") >> "$out" || exit 1
    echo "pair $i tree $t done ($(date +%T))"
  done
done
