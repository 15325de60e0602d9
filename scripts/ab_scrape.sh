cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in 1 2 3; do
  for t in . ab_old; do
    (cd $t && timeout -k 10 120 python scripts/scrape_probe.py 2>/dev/null | tail -1 | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('$t', 'c1', d['threads2_conns1']['rps'], d['threads2_conns1']['p50_us'], 'c2', d['threads2_conns2']['rps'], 'c4', d['threads4_conns4']['rps'], 'bytes', d['threads2_conns1']['bytes'], 'render', d['render_ns_threads1'])") >> gpurun_out/ab_scrape.txt || exit 1
  done
done
