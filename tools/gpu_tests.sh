#!/bin/bash
# run the given GPU test files in ONE pytest process on the GPU box (log under gpurun_out/), e.g.
#   gpurun -- 'bash tools/gpu_tests.sh tests/test_iq_grid.py'
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 ${GPU_TEST_TIMEOUT:-500} python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread "$@" \
    > gpurun_out/tests.log 2>&1
rc=$?
tail -5 gpurun_out/tests.log
exit $rc
