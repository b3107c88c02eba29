#!/bin/bash
# round-4 GPU session B: the whole GPU suite, then the bench line (defaults, with the CPU baseline) and the prefill
# PMC passes.  Logs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
GPU_TEST_TIMEOUT=800 bash tools/gpu_tests.sh tests/ || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r04.log 2>&1 || exit $?
tail -1 gpurun_out/bench_r04.log
