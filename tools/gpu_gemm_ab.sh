#!/bin/bash
# Q4_K prefill GEMM A/B at ubatch 512 (tools/gemm_ab.py): default dispatch vs v5 with 2 / 3 / 4 K ranges
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for sh in qkv wo down; do
  GEMM_ONLY=$sh timeout -k 10 200 python3 tools/gemm_ab.py 0 21 22 23 >> gpurun_out/gemm_ab_r5.log 2>&1 || exit $?
done
