#!/bin/bash
# r5: three bench runs (tail attribution + batched floor), then the 1 s-idle probe with
# per-segment attribution from the daemon's call trace.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$PWD/gpurun_out/r5"
mkdir -p "$OUT"
for tag in a b c; do
  echo "=== bench $tag ($(date +%T))"
  timeout -k 10 300 python bench.py > "$OUT/bench_$tag.log" 2>&1 || exit $?
  tail -1 "$OUT/bench_$tag.log" | cut -c1-200
done
echo "=== idle probe ($(date +%T))"
timeout -k 10 700 python -u scripts/idle_probe.py --gaps ${IDLE_GAPS:-0.001,1} --calls ${IDLE_CALLS:-80} \
  --out "$OUT/idle_probe_segments.json" > "$OUT/idle_probe.log" 2>&1 || exit $?
grep attribution "$OUT/idle_probe.log" | cut -c1-1500
echo "=== done"
