#!/bin/bash
# Q8_0 tile GEMM: per shape, weights cold (8 copies rotated past the Infinity Cache) vs warm (one copy, IC-resident)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for sh in qkv wo down gate_up; do
  timeout -k 10 120 python3 tools/q80t_shapes.py $sh >> gpurun_out/q80t_ab.log 2>/dev/null || exit $?
  timeout -k 10 120 python3 tools/q80t_shapes.py $sh --warm >> gpurun_out/q80t_ab.log 2>/dev/null || exit $?
done
