#!/bin/bash
# Interleaved A/B of two daemon configs on one lease: bench.py runs A B A B ..., no canary.
# Usage: scripts/r6_ab.sh <tag> '<json A>' '<json B>' [pairs]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=$1; A=$2; B=$3; pairs=${4:-2}
out=gpurun_out/r6
mkdir -p $out
for i in $(seq 1 $pairs); do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-canary --daemon-config "$A" > $out/ab_${tag}_A_$i.json 2> $out/ab_${tag}_A_$i.err || exit 1
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-canary --daemon-config "$B" > $out/ab_${tag}_B_$i.json 2> $out/ab_${tag}_B_$i.err || exit 1
done
echo ab done
