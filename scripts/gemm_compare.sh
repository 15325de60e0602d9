mkdir -p gpurun_out && export PYTHONPATH=$PWD
[ -n "$NOTEST" ] || timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu.py -k "lds_gemm" -s > gpurun_out/g256_test.log 2>&1
for sz in 4096 8192; do
  it=$(( sz == 4096 ? 400 : 60 ))
  for kk in ${KERNELS:-lds128 pingpong256 pingpong256s}; do
    timeout -k 10 60 python -m k8s_gpu_device_plugin_amd.ops.canary --gemm $sz --gemm-iters $it --gemm-kernel $kk --gemm-random || exit 1
  done
  timeout -k 10 90 python -c "
import torch,time,json;n=$sz;x=torch.rand(n,n,device='cuda',dtype=torch.bfloat16)*2-1;y=torch.rand(n,n,device='cuda',dtype=torch.bfloat16)*2-1
[x@y for _ in range(10)];torch.cuda.synchronize();t=time.perf_counter();[x@y for _ in range($it)];torch.cuda.synchronize()
print(json.dumps({'torch_matmul_tflops':2*n**3*$it/(time.perf_counter()-t)/1e12,'shape':n,'iters':$it}))" || exit 1
done
