#!/bin/bash
# after the Q5_K GLU rule: GEMM / MoE tests, Mixtral bench, headline bench (prefill line included)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rs.py tests/test_gpu_kernels.py tests/test_gpu_moe.py tests/test_gpu_moe_fullwidth.py > gpurun_out/glu2_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --config mixtral-8x7b-q5_k_m --steps 32 --warmup 4 --no-cpu-baseline > gpurun_out/glu2_mix.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/glu2_bench.log 2>&1 || exit $?
