#!/bin/bash
# round-5 GPU session E: fused rope/KV q|k|v epilogue, key-split + TA attention, Q8_0 tile GEMM variants, config 3
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
[ -n "$SKIP_UNIT" ] || timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_q80t.py tests/test_gpu_fa_split.py > gpurun_out/r5e_unit.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_rowsplit.py tests/test_gpu_fullsize.py -k "q8_0 or Q8_0 or rowsplit or legacy or fused_decode" > gpurun_out/r5e_model.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config llama3-8b-q8_0-b32 --steps 32 --warmup 4 > gpurun_out/r5e_cfg3.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5e_cfg3 -o run -- python3 bench.py --config llama3-8b-q8_0-b32 --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/r5e_cfg3_prof.log 2>&1 || exit $?
for v in "" _v2; do
  [ -f koboldcpp_amd/koboldcpp_hipblas$v.so ] || continue
  KCPP_LIB=$PWD/koboldcpp_amd/koboldcpp_hipblas$v.so timeout -k 10 500 python3 tools/q80t_sweep.py --full > gpurun_out/q80t$v.log 2>&1 || exit $?
done
