#!/bin/bash
# Q5_K on the int8 v4 GEMM: bitwise vs v2 + the Q5_K GEMM / MoE tests, then timing v2 (2) vs v4 (0) at the Mixtral
# expert shapes (M = 128: ubatch 512 top-2 over 8 experts) and M = 512
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rs.py -k "v4_int8" > gpurun_out/q5v4_bitwise.log 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "Q5_K or 13 or mul_mat or gemm" > gpurun_out/q5v4_kernels.log 2>&1 || exit $?
for m in 128 512; do
  GEMM_M=$m GEMM_ONLY=glu5 timeout -k 10 120 python3 tools/gemm_ab.py 2 0 >> gpurun_out/q5v4_ab.log 2>&1 || exit $?
  GEMM_M=$m GEMM_ONLY=down5 timeout -k 10 120 python3 tools/gemm_ab.py 2 0 >> gpurun_out/q5v4_ab.log 2>&1 || exit $?
  GEMM_M=$m GEMM_ONLY=wo5 timeout -k 10 120 python3 tools/gemm_ab.py 2 0 >> gpurun_out/q5v4_ab.log 2>&1 || exit $?
  GEMM_M=$m GEMM_ONLY=glu5rs timeout -k 10 120 python3 tools/gemm_ab.py 2 0 >> gpurun_out/q5v4_ab.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_moe.py tests/test_gpu_moe_fullwidth.py > gpurun_out/q5v4_moe.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --config mixtral-8x7b-q5_k_m --steps 32 --warmup 4 --no-cpu-baseline > gpurun_out/q5v4_mix.log 2>&1 || exit $?
