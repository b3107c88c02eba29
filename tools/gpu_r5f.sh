#!/bin/bash
# round-5 GPU session F: Q8_0 tile path (GLU on the ring loop, merged-split attention), tests, config 3 bench + profile
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_q80t.py tests/test_gpu_fa_split.py > gpurun_out/r5f_unit.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_rowsplit.py tests/test_gpu_fullsize.py -k "q8_0 or Q8_0 or rowsplit or legacy or fused_decode" > gpurun_out/r5f_model.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config llama3-8b-q8_0-b32 --steps 32 --warmup 4 > gpurun_out/r5f_cfg3.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5f_cfg3 -o run -- python3 bench.py --config llama3-8b-q8_0-b32 --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/r5f_cfg3_prof.log 2>&1 || exit $?
