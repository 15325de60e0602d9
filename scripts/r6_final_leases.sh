#!/bin/bash
# r6: the final tree on one more lease - three bench runs as the driver runs them (with the
# canary), each carrying its host fingerprint, placement and paired floor.
# Usage: scripts/r6_final_leases.sh <tag>   (outputs under gpurun_out/r6/)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-final}
out=gpurun_out/r6
mkdir -p $out
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $out/bench_${tag}_$i.json 2> $out/bench_${tag}_$i.err || exit 1
  python3 -c "
import json
d = json.loads(open('$out/bench_${tag}_$i.json').read().strip().splitlines()[-1])
p = d['allocate_vs_spin_floor_paired']
print(json.dumps({'p50': d['value'], 'floor_spin': d['uds_roundtrip_floor_spin_p50_us'], 'paired': p['ratio_median'],
                  'ci': p['ratio_ci95'], 'p999': d['allocate_p999_us'], 'load': d['host'].get('loadavg')}))"
done
echo leases done
