#!/bin/bash
# 8-rank bench.py rehearsal (gloo ranks on the CPU, GPUs hidden from them) against an
# 8-GPU fixture daemon: the driver's N=8 path (16 gRPC and 16 HTTP workers, 8 clients).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
HIP_VISIBLE_DEVICES=-1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29788 bench.py --gpus 8 --steps 10 --warmup 2 --backend fixture \
  > gpurun_out/rehearse_n8.log 2>&1 || { echo "n=8 failed"; tail -20 gpurun_out/rehearse_n8.log; exit 1; }
grep '^{' gpurun_out/rehearse_n8.log | tail -1 | cut -c1-300
