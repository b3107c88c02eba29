#!/bin/bash
# Q8_0 tile GEMM: shape sweep (tools/q80t_sweep.py), its tests, config 3 bench line
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/q80t_sweep.py > gpurun_out/q80t_v1.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_q80t.py > gpurun_out/r5d_q80t.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config llama3-8b-q8_0-b32 --steps 32 --warmup 4 > gpurun_out/r5d_cfg3.log 2>&1 || exit $?
