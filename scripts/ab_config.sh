#!/bin/bash
# A/B of bench.py between daemon configurations on one box, interleaved: ARMS is a list of
# "name=JSON" config overrides (bench.py --daemon-config), PAIRS rounds in rotating order.
# Each line: arm, Allocate p50, p99, polling floor p50, cold p50, admission p50, /metrics
# RPS, /metrics p50.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out="gpurun_out/${AB_OUT:-ab_config.txt}"
mapfile -t arms < <(printf '%s\n' "${ARMS[@]:-}" | tr ';' '\n' | sed '/^$/d')
[ ${#arms[@]} -gt 0 ] || { echo "ARMS='a={...};b={...}'"; exit 2; }
for i in $(seq 1 ${PAIRS:-5}); do
  k=${#arms[@]}
  for j in $(seq 0 $((k - 1))); do
    arm=${arms[$(( (i + j) % k ))]}
    name=${arm%%=*}; cfg=${arm#*=}
    timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-canary --daemon-config "$cfg" 2>/dev/null | tail -1 | python -c "
import json, sys
d = json.loads(sys.stdin.read())
print('$name', d['value'], d['allocate_p99_us'], d['uds_roundtrip_floor_spin_p50_us'], d['allocate_cold_p50_us'],
      d['allocate_admission_p50_us'], d['scrape_rps'], d['scrape_p50_us'])" >> "$out" || exit 1
    echo "pair $i arm $name done ($(date +%T))"
  done
done
