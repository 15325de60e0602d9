#!/bin/bash
# r5: the current build against a variant build of the native module (AB_SO, loaded by
# the bench and its daemon through AMDGPU_DP_NATIVE_SO), alternated three times.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$PWD/gpurun_out/r5"
mkdir -p "$OUT"
: > "$OUT/ab_variant.jsonl"
for i in 1 2 3; do
  for arm in cur variant; do
    echo "=== bench $arm #$i ($(date +%T))"
    if [ $arm = variant ]; then export AMDGPU_DP_NATIVE_SO="$PWD/$AB_SO"; else unset AMDGPU_DP_NATIVE_SO; fi
    timeout -k 10 300 python bench.py > "$OUT/bench_ab_$arm.log" 2>&1 || exit $?
    tail -1 "$OUT/bench_ab_$arm.log" | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print(json.dumps({'arm': '$arm', 'round': $i, 'p50': d['value'], 'floor_spin': d['uds_roundtrip_floor_spin_p50_us'],
                  'pref': d['preferred_p50_us'], 'pref_server': d.get('preferred_server_mean_us'),
                  'alloc_server': d['allocate_server_mean_us'], 'admission': d['allocate_admission_p50_us'],
                  'p999': d['allocate_p999_us'], 'scrape_p50': d['scrape_p50_us']}))" | tee -a "$OUT/ab_variant.jsonl"
  done
done
echo "=== done"
