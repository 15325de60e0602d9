#!/bin/bash
# Multi-rank bench.py rehearsal without N GPUs: ranks on the CPU (gloo, GPUs hidden from
# the ranks), daemon on an N-GPU fixture node (bench.py refuses to report N GPUs that
# the daemon did not advertise, so a 1-GPU amdsmi daemon cannot serve N ranks).
# Exercises the N>1 driver path: rendezvous, rank r -> device r, barriers, the gather.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for n in 2 4; do
  HIP_VISIBLE_DEVICES=-1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29700 + n)) bench.py --gpus $n --steps 10 --warmup 2 --backend fixture \
    > gpurun_out/rehearse_n$n.log 2>&1 || { echo "n=$n failed"; tail -20 gpurun_out/rehearse_n$n.log; exit 1; }
  tail -1 gpurun_out/rehearse_n$n.log | cut -c1-400
done
