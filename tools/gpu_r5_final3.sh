#!/bin/bash
# round-5 close (after the grouped MoE / Q5_K rule changes): shape check, whole GPU suite, smoke(), bench lines
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for sh in gu5 qkv5 down5 wo5; do
  GEMM_M=128 GEMM_ONLY=$sh timeout -k 10 120 python3 tools/gemm_ab.py 2 0 >> gpurun_out/f3_shapes.log 2>&1 || exit $?
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/f3_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/f3_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/f3_bench.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --config mixtral-8x7b-q5_k_m --steps 32 --warmup 4 --no-cpu-baseline > gpurun_out/f3_mix.log 2>&1 || exit $?
