#!/bin/bash
# Q8_0 tile GEMM: its tests, (S, WV) grid for the built-in loop and the ring variant (KCPP_LIB builds), model-level
# Q8_0 tests, config 3 bench
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_q80t.py > gpurun_out/r5d_q80t.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_rowsplit.py tests/test_gpu_fullsize.py -k "q8_0 or Q8_0 or rowsplit or legacy or fused_decode" > gpurun_out/r5d_model.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config llama3-8b-q8_0-b32 --steps 32 --warmup 4 > gpurun_out/r5d_cfg3.log 2>&1 || exit $?
for v in "" _v2 _v3; do
  [ -f koboldcpp_amd/koboldcpp_hipblas$v.so ] || continue
  KCPP_LIB=$PWD/koboldcpp_amd/koboldcpp_hipblas$v.so timeout -k 10 500 python3 tools/q80t_sweep.py --full > gpurun_out/q80t$v.log 2>&1 || exit $?
done
