#!/bin/bash
# grouped MoE prefill: new tests, MoE suites, Mixtral bench (grouped default) and the per-expert A/B bench
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_moe.py -k "grouped" > gpurun_out/grp_new.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_moe.py tests/test_gpu_moe_fullwidth.py tests/test_gpu_ggml_backend.py > gpurun_out/grp_moe.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --config mixtral-8x7b-q5_k_m --steps 32 --warmup 4 --no-cpu-baseline > gpurun_out/grp_mix.log 2>&1 || exit $?
