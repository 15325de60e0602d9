#!/bin/bash
# Multi-rank bench.py rehearsal without N GPUs: ranks on the CPU (gloo, GPUs hidden from
# the ranks), daemon on an N-GPU fixture node (bench.py refuses to report N GPUs that
# the daemon did not advertise, so a 1-GPU amdsmi daemon cannot serve N ranks).
# Exercises the N>1 driver path: rendezvous, rank -> the device whose hip_id is its
# local rank, barriers, the gather.  RANKS (default "2 4 8") picks the sizes; PERMUTED=1
# also runs 4 ranks on a node whose HIP ordinals are permuted against BDF order.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {  # run <n> <tag> [fixture]
  local n=$1 tag=$2 fx=${3:-}
  HIP_VISIBLE_DEVICES=-1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29700 + n)) bench.py --gpus $n --steps 10 --warmup 2 --backend fixture \
    ${fx:+--fixture $fx} > gpurun_out/rehearse_$tag.log 2>&1 || { echo "$tag failed"; tail -20 gpurun_out/rehearse_$tag.log; exit 1; }
  tail -1 gpurun_out/rehearse_$tag.log > gpurun_out/rehearse_$tag.json
  cut -c1-400 gpurun_out/rehearse_$tag.json
}
for n in ${RANKS:-2 4 8}; do run $n n$n; done
if [ "${PERMUTED:-1}" = 1 ]; then run 4 n4_hip_permuted 4gpu_spx_hip_permuted; fi
