#!/bin/bash
# Multi-rank bench.py rehearsal on a 1-GPU box: ranks on the CPU (gloo, GPUs hidden from
# the ranks), daemon on the real amdsmi backend.  Exercises the N>1 driver path.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for n in 2 4; do
  HIP_VISIBLE_DEVICES=-1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29700 + n)) bench.py --gpus $n --steps 10 --warmup 2 \
    > gpurun_out/rehearse_n$n.log 2>&1 || { echo "n=$n failed"; tail -20 gpurun_out/rehearse_n$n.log; exit 1; }
  tail -1 gpurun_out/rehearse_n$n.log | cut -c1-400
done
