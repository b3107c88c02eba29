#!/bin/bash
# the asm-DMA staging in q4v3 (parity tests), the 3-stage Q8_0 ring A/B (config 3), q4v3 before / after at M = 32
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_rs.py tests/test_gpu_kernels.py tests/test_gpu_production_vs_oracle.py tests/test_gpu_fullsize.py > gpurun_out/q80b_tests.log 2>&1 || { tail -5 gpurun_out/q80b_tests.log; exit 1; }
tail -1 gpurun_out/q80b_tests.log
for lib in koboldcpp_hipblas koboldcpp_hipblas_st3; do
  KCPP_LIB=$PWD/koboldcpp_amd/$lib.so timeout -k 10 300 python -u bench.py --config llama3-8b-q8_0-b32 --no-cpu-baseline > gpurun_out/cfg3_$lib.log 2>&1 || exit $?
  echo "$lib $(tail -1 gpurun_out/cfg3_$lib.log | cut -c60-120)"
  for sh in "gate|up" qkv down; do KCPP_LIB=$PWD/koboldcpp_amd/$lib.so GEMM_M=32 GEMM_ONLY="$sh" timeout -k 10 200 python -u tools/gemm_ab.py 0 | sed "s/^/$lib /" || exit $?; done
done
