#!/bin/bash
# r6: grpc.coreEscape off / on, alternated on one lease, bench.py as the driver runs it.
# Usage: scripts/r6_escape_ab.sh <tag> [pairs]   (outputs under gpurun_out/r6/)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-esc}
out=gpurun_out/r6
mkdir -p $out
for i in $(seq 1 ${2:-3}); do
  for arm in off on; do
    flag=false; [ $arm = on ] && flag=true
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --daemon-config "{\"grpc\": {\"coreEscape\": $flag}}" \
      > $out/bench_${tag}_${arm}_$i.json 2> $out/bench_${tag}_${arm}_$i.err || exit 1
    python3 -c "
import json
d = json.loads(open('$out/bench_${tag}_${arm}_$i.json').read().strip().splitlines()[-1])
r = d['placement']['allocate_by_relation']
print('$arm', d['value'], d['allocate_vs_spin_floor_paired']['ratio_median'], {k: (v['calls'], v['p50_us']) for k, v in r.items() if k not in ('pairs', 'batch_p50_us')})"
  done
done
echo ab done
