#!/bin/bash
# Q5_K dense gate|up (one 4096 x 28672 GEMM, mode 0) and q|k|v: v2 (2) vs default (0)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for m in 128 512 512; do
  for sh in gu5 qkv5; do
    GEMM_M=$m GEMM_ONLY=$sh timeout -k 10 120 python3 tools/gemm_ab.py 2 0 2 0 >> gpurun_out/gu5.log 2>&1 || exit $?
  done
done
