#!/bin/bash
# grouped expert GEMM tile-shape A/B + the grouped tests
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/grouped_ab.py 0 15 17 0 > gpurun_out/gab.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_moe.py -k grouped > gpurun_out/gab_tests.log 2>&1 || exit $?
