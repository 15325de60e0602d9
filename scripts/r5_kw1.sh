#!/bin/bash
# r5: keepWarmMs 1 as the default - bench twice, a replicated 1 s A/B against 10 ms (two
# daemons per setting, calls interleaved), and the idle probe over 1 ms .. 1 s gaps.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$PWD/gpurun_out/r5"
mkdir -p "$OUT"
for tag in kw1a kw1b; do
  echo "=== bench $tag ($(date +%T))"
  timeout -k 10 300 python bench.py > "$OUT/bench_$tag.log" 2>&1 || exit $?
  tail -1 "$OUT/bench_$tag.log" | cut -c1-160
done
echo "=== idle A/B x2 ($(date +%T))"
timeout -k 10 600 python -u scripts/idle_probe.py --gaps 1 --calls 60 --rpcs allocate --replicas 2 \
  --ab-overrides '{"kw1": {"grpc": {"keepWarmMs": 1}}, "kw10": {"grpc": {"keepWarmMs": 10}}}' \
  --out "$OUT/idle_ab_kw1_vs_10_x2.json" > "$OUT/idle_ab_x2.log" 2>&1 || exit $?
grep -v progress "$OUT/idle_ab_x2.log" | tail -1 | cut -c1-600
echo "=== idle gaps ($(date +%T))"
timeout -k 10 700 python -u scripts/idle_probe.py --gaps 0.001,0.01,0.1,1 --calls 60 \
  --out "$OUT/idle_probe_gaps_kw1.json" > "$OUT/idle_gaps.log" 2>&1 || exit $?
grep attribution "$OUT/idle_gaps.log" | cut -c1-1500
echo "=== done"
