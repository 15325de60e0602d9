cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/placement_probe.txt
python -c "import os; a=sorted(os.sched_getaffinity(0)); print('affinity', len(a), a[:4], a[-4:])" > $out
cat /sys/devices/system/cpu/cpu0/cache/index3/shared_cpu_list >> $out 2>&1
cat /sys/devices/system/cpu/cpu0/topology/thread_siblings_list >> $out 2>&1
lscpu | grep -E "NUMA node|Socket|Thread|Core|L3" >> $out 2>&1
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-canary 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('free', d['value'], d['allocate_p99_us'], d['uds_roundtrip_floor_spin_p50_us'])" >> $out || exit 1
  timeout -k 10 120 taskset -c 0-7 python bench.py --steps 20 --warmup 5 --no-canary 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('llc0', d['value'], d['allocate_p99_us'], d['uds_roundtrip_floor_spin_p50_us'])" >> $out || exit 1
done
