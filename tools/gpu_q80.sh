#!/bin/bash
# Q8_0 small-batch GEMM / Q6_K GEMM staging change: parity tests, config 3, the Q6_K GEMM A/B shapes, the bench line
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_rs.py tests/test_gpu_production_vs_oracle.py tests/test_gpu_fullsize.py > gpurun_out/q80_tests.log 2>&1
rc=$?; tail -2 gpurun_out/q80_tests.log; [ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
timeout -k 10 300 python -u bench.py --config llama3-8b-q8_0-b32 --no-cpu-baseline > gpurun_out/cfg3.log 2>&1 || exit $?
tail -1 gpurun_out/cfg3.log | cut -c1-200
for sh in down6 v6; do GEMM_ONLY=$sh timeout -k 10 200 python -u tools/gemm_ab.py 0 || exit $?; done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_q80.log 2>&1 || exit $?
grep -o '"value": [0-9.]*\|"prefill_tok_s": [0-9.]*' gpurun_out/bench_q80.log | head -2
