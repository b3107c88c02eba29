#!/bin/bash
# after the Q5_K rule change: shapes (default should now match v2 where unsplit), GEMM / MoE tests, Mixtral bench
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for sh in gu5 qkv5 down5 wo5; do
  GEMM_M=128 GEMM_ONLY=$sh timeout -k 10 120 python3 tools/gemm_ab.py 2 0 >> gpurun_out/gu5b.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rs.py tests/test_gpu_kernels.py tests/test_gpu_moe.py tests/test_gpu_ggml_backend.py > gpurun_out/gu5b_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --config mixtral-8x7b-q5_k_m --steps 32 --warmup 4 --no-cpu-baseline > gpurun_out/gu5b_mix.log 2>&1 || exit $?
