#!/bin/bash
# end-of-round check: the whole GPU suite, smoke(), and the default bench line (with the CPU baseline)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
GPU_TEST_TIMEOUT=800 bash tools/gpu_tests.sh tests/ || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit $?
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_final.log 2>&1 || exit $?
tail -1 gpurun_out/bench_final.log | cut -c1-300
