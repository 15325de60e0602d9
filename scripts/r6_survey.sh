#!/bin/bash
# Round-6 survey on one lease: host fingerprint + placement of several bench runs, the
# admission window A/B (bench first-of-batch, 1 s idle probe) and the idle daemon's cost.
# Usage: scripts/r6_survey.sh <tag>   (outputs under gpurun_out/r6/)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-lease}
out=gpurun_out/r6
mkdir -p $out
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-canary > $out/bench_${tag}_$i.json 2> $out/bench_${tag}_$i.err || exit 1
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-canary --daemon-config '{"grpc": {"activeWindowMs": 0}}' \
  > $out/bench_${tag}_always.json 2> $out/bench_${tag}_always.err || exit 1
timeout -k 10 120 python scripts/idle_wakeups.py --out $out/idle_wakeups_${tag}.json > $out/idle_wakeups_${tag}.log 2>&1 || exit 1
timeout -k 10 120 python scripts/idle_wakeups.py --daemon-config '{"grpc": {"activeWindowMs": 0}}' \
  --out $out/idle_wakeups_${tag}_always.json > $out/idle_wakeups_${tag}_always.log 2>&1 || exit 1
if [ "${IDLE_AB:-1}" = 1 ]; then
  timeout -k 10 400 python scripts/idle_probe.py --gaps 1 --calls 40 --rpcs allocate \
    --ab-overrides '{"window10s": {}, "always": {"grpc": {"activeWindowMs": 0}}}' \
    --out $out/idle_ab_window_${tag}.json > $out/idle_ab_window_${tag}.log 2>&1 || exit 1
fi
echo survey done
