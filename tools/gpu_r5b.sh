#!/bin/bash
# round-5 GPU session B: long-K RS decode (70B ffn_down), the tests around it, the generate() leg and the 70B stage
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_production_vs_oracle.py tests/test_gpu_config4.py tests/test_gpu_rs.py tests/test_gpu_moe.py tests/test_gpu_moe_fullwidth.py tests/test_gpu_expose.py > gpurun_out/r5b_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 64 --warmup 8 --no-cpu-baseline > gpurun_out/r5b_bench.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --config llama3-70b-stage --steps 64 --warmup 8 > gpurun_out/r5b_70b.log 2>&1 || exit $?
