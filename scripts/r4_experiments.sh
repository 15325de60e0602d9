#!/bin/bash
# Round-4 measurements on one box (one gpurun call): the scrape-path A/B across the
# round-2, round-3 and current trees, then the idle-gap probe with
# the daemon's own time per call, keep-warm off and on (item 6).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD:$PYTHONPATH"
mkdir -p gpurun_out
TREES=". ab_r3 ab_r2" PAIRS=${PAIRS:-3} AB_OUT=ab_scrape_r2_r3_r4.txt bash scripts/ab_tree.sh || exit $?
for kw in 0 10; do
  timeout -k 10 500 python -u scripts/idle_probe.py --gaps 1 --calls ${CALLS:-100} --server-time --keep-warm-ms $kw \
    --out gpurun_out/idle_probe_1s_keepwarm$kw.json > gpurun_out/idle_probe_1s_keepwarm$kw.log 2>&1 || exit $?
  tail -1 gpurun_out/idle_probe_1s_keepwarm$kw.log | cut -c1-1500
done
