#!/bin/bash
# Q8_0 tile GEMM A/B: per-shape timing (tools/q80t_shapes.py) for the default build and KCPP_LIB variants, + the
# variant's tests
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in "" _v2; do
  [ -f koboldcpp_amd/koboldcpp_hipblas$v.so ] || continue
  for sh in gate_up gate_up; do
    KCPP_LIB=$PWD/koboldcpp_amd/koboldcpp_hipblas$v.so timeout -k 10 120 python3 tools/q80t_shapes.py $sh >> gpurun_out/q80t_ab$v.log 2>/dev/null || exit $?
  done
done
KCPP_LIB=$PWD/koboldcpp_amd/koboldcpp_hipblas_v2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_q80t.py > gpurun_out/q80t_ab_tests.log 2>&1 || exit $?
