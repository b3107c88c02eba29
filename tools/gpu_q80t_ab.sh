#!/bin/bash
# Q8_0 tile GEMM: per-shape timing (tools/q80t_shapes.py) + its tests
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for sh in qkv wo down gate_up; do
  timeout -k 10 120 python3 tools/q80t_shapes.py $sh >> gpurun_out/q80t_ab.log 2>/dev/null || exit $?
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_q80t.py > gpurun_out/q80t_ab_tests.log 2>&1 || exit $?
