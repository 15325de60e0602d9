#!/bin/bash
# Keep-warm A/B on one box (one gpurun call): the first Allocate after 1 s idle, minus a
# bare unix-socket exchange after the same gap, for three daemon settings - the full
# in-memory request path (grpc.keepWarmFull true), HPACK + table only (false), and off
# (keepWarmMs 0) - two daemons each, calls interleaved (scripts/idle_probe.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 850 python -u scripts/idle_probe.py --gaps 1 --calls ${CALLS:-100} --replicas ${REPLICAS:-2} --rpcs allocate \
  --ab-overrides '{"full": {"grpc": {"keepWarmFull": true}}, "table": {"grpc": {"keepWarmFull": false}}, "off": {"grpc": {"keepWarmMs": 0}}}' \
  --out gpurun_out/idle_ab_keepwarm_full_table_off.json > gpurun_out/idle_ab_kw_full.log 2>&1
