#!/bin/bash
# round-5 end: Q8_0 / attention / MoE unit tests, the default bench line, config 3
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_q80t.py tests/test_gpu_fa_split.py tests/test_gpu_moe.py tests/test_gpu_model.py > gpurun_out/r5_end_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/r5_end_bench.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config llama3-8b-q8_0-b32 --steps 32 --warmup 4 > gpurun_out/r5_end_cfg3.log 2>&1 || exit $?
