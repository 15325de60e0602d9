cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for bp in 0 50 0 50 0 50; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-canary --busy-poll-us $bp > gpurun_out/ab_$bp.json.tmp 2>gpurun_out/ab_err.log || exit $?
  grep '^{' gpurun_out/ab_$bp.json.tmp >> gpurun_out/ab_$bp.jsonl
done
