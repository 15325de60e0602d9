#!/bin/bash
# r5: final tree - the final check (GPU tests, smoke, bench x3), then a 300 s amdsmi soak.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$PWD/gpurun_out/r5"
bash scripts/r5_final_check.sh || exit $?
echo "=== soak 300 s ($(date +%T))"
timeout -k 10 420 python -u scripts/soak.py --seconds 300 --backend amdsmi > "$OUT/soak_final.log" 2>&1 || exit $?
tail -1 "$OUT/soak_final.log" | cut -c1-700
echo "=== done"
