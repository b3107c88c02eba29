#!/bin/bash
# round-5 GPU session C: generate() device-token fast path -- the drop-in ABI tests and the bench's generate() leg
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_expose.py tests/test_gpu_context_shift.py > gpurun_out/r5c_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 64 --warmup 8 --no-cpu-baseline > gpurun_out/r5c_bench.log 2>&1 || exit $?
