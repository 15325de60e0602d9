#!/bin/bash
# r5: 1 s-idle Allocate, three keep-warm settings interleaved call by call (one daemon
# each), with the daemon's per-call segments; one bench run for the record.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$PWD/gpurun_out/r5"
mkdir -p "$OUT"
echo "=== idle A/B ($(date +%T))"
timeout -k 10 600 python -u scripts/idle_probe.py --gaps 1 --calls ${IDLE_CALLS:-60} --rpcs allocate \
  --ab-overrides '{"kw10": {"grpc": {"keepWarmMs": 10}}, "kw1": {"grpc": {"keepWarmMs": 1}}, "kw0": {"grpc": {"keepWarmMs": 0}}}' \
  --out "$OUT/idle_ab_kw_10_1_0.json" > "$OUT/idle_ab.log" 2>&1 || exit $?
grep -v progress "$OUT/idle_ab.log" | tail -2 | cut -c1-3000
echo "=== done"
