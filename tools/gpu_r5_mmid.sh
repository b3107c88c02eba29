#!/bin/bash
# ggml-backend MUL_MAT_ID on the grouped GEMM: backend + MoE suites
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ggml_backend.py tests/test_gpu_moe.py tests/test_gpu_moe_fullwidth.py tests/test_gpu_expose.py > gpurun_out/mmid_tests.log 2>&1 || exit $?
