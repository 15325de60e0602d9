#!/bin/bash
# r5: /metrics after the header-parsing and histogram-shard changes: bench.py three times
# (scrape RPS, p50, the daemon's own time per scrape against the TCP floor).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$PWD/gpurun_out/r5"
mkdir -p "$OUT"
: > "$OUT/http_bench.jsonl"
for i in 1 2 3; do
  echo "=== bench #$i ($(date +%T))"
  timeout -k 10 300 python bench.py > "$OUT/bench_http_$i.log" 2>&1 || exit $?
  tail -1 "$OUT/bench_http_$i.log" | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print(json.dumps({'round': $i, 'p50': d['value'], 'p99': d['allocate_p99_us'], 'p999': d['allocate_p999_us'],
                  'scrape_rps': d['scrape_rps'], 'scrape_p50': d['scrape_p50_us'], 'scrape_p99': d['scrape_p99_us'],
                  'scrape_server_mean': d['scrape_server_mean_us'], 'tcp_floor': d['tcp_scrape_floor_p50_us'],
                  'metrics_bytes': d['metrics_bytes'], 'other': d['allocate_tail']['other']}))" | tee -a "$OUT/http_bench.jsonl"
done
echo "=== done"
