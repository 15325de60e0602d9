# A/B of scripts/concurrency_probe.py between this tree (.) and ./ab_old, alternating on one box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in 1 2; do
  for t in . ab_old; do
    (cd $t && timeout -k 10 240 python scripts/concurrency_probe.py --clients ${CLIENTS:-2,4,8,16} 2>/dev/null | sed "s|^|$t |") >> gpurun_out/ab_concurrency.txt || exit 1
  done
done
