#!/bin/bash
# One gpurun call: GPU tests, smoke, bench, rocprof of the canary kernels.
# Ordinary test failures (rc 1) do not stop the script; faults/timeouts/aborts do.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD:$PYTHONPATH"
OUT="$PWD/gpurun_out"
mkdir -p "$OUT"
step() {  # step <name> <timeout> <cmd...>
  local name=$1 tmo=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "=== stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in ${STEPS:-pytest smoke bench prof}; do
  case $s in
    pytest) step pytest_gpu 420 python -u -m pytest tests -x -v -m gpu -s -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    smoke)  step smoke 240 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  step bench 300 python bench.py ${BENCH_ARGS:-} ;;
    idle)   step idle_probe ${IDLE_TIMEOUT:-400} python -u scripts/idle_probe.py --gaps ${IDLE_GAPS:-0.001,0.01,0.1} --calls ${IDLE_CALLS:-300} --out "$OUT/idle_probe${IDLE_TAG:-}.json" ;;
    soak)   step soak $(( ${SOAK_SECONDS:-120} + 120 )) python -u scripts/soak.py --seconds ${SOAK_SECONDS:-120} --backend amdsmi ;;
    suite)  step suite 600 python -m k8s_gpu_device_plugin_amd.benchmark.suite --json "$OUT/baseline_suite_gpu.json" ;;
    sweep)  step hbm_sweep 300 python -c "import json; from k8s_gpu_device_plugin_amd.ops import canary; rows = canary.hbm_sweep(0); print(json.dumps(rows, indent=1)); json.dump(rows, open('$OUT/hbm_sweep.json', 'w'), indent=1)" ;;
    prof)   (cd /tmp && export TMPDIR=/tmp && step rocprof_canary 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof_canary" -o canary --output-format csv -- python3 -m k8s_gpu_device_plugin_amd.ops.canary --device 0 --bytes 2147483648 --passes 3) ;;
    pmc)    # one derived counter per pass ("exceeds the capabilities" otherwise); short limits
            # PMC_CTRS="A;B C" overrides the list (';' separates passes)
            IFS=';' read -r -a ctrs <<< "${PMC_CTRS:-FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES}"
            for ctr in "${ctrs[@]}"; do
              tag=$(echo "$ctr" | tr ' ' '_')
              (cd /tmp && export TMPDIR=/tmp && step "pmc_$tag" 90 rocprofv3 --pmc $ctr --kernel-trace --stats -d "$OUT/pmc_$tag" -o canary --output-format csv -- python3 -m k8s_gpu_device_plugin_amd.ops.canary --device 0 --bytes 1073741824 --passes 1) || exit $?
            done ;;
    gemmprof)  # matrix-path canary kernel: trace + one PMC group per pass
            (cd /tmp && export TMPDIR=/tmp && step rocprof_gemm 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof_gemm" -o gemm --output-format csv -- python3 -m k8s_gpu_device_plugin_amd.ops.canary ${GEMM_ARGS:---gemm 4096}) || exit $?
            IFS=';' read -r -a ctrs <<< "${GEMM_PMC:-SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_ADDR_CONFLICT;SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16;FETCH_SIZE;GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY}"
            for ctr in "${ctrs[@]}"; do
              tag=$(echo "$ctr" | tr ' ' '_')
              (cd /tmp && export TMPDIR=/tmp && step "gemm_pmc_$tag" 90 rocprofv3 --pmc $ctr --kernel-trace --stats -d "$OUT/gemm_pmc_$tag" -o gemm --output-format csv -- python3 -m k8s_gpu_device_plugin_amd.ops.canary ${GEMM_ARGS:---gemm 4096} --gemm-iters 5) || exit $?
            done ;;
  esac
done
echo "=== done"
