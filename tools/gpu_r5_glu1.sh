#!/bin/bash
# v4 GLU as one launch (gate + up): bitwise tests, then v2 (2) / default (0) / forced v4 (13) at the expert GLU shapes
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rs.py -k "v4_int8 or v5" > gpurun_out/glu1_bitwise.log 2>&1 || exit $?
for m in 128 512; do
  for sh in glu5 glu2 glu5 glu2; do
    GEMM_M=$m GEMM_ONLY=$sh timeout -k 10 120 python3 tools/gemm_ab.py 2 0 13 >> gpurun_out/glu1_ab.log 2>&1 || exit $?
  done
done
