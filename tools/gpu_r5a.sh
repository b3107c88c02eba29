#!/bin/bash
# round-5 GPU session A: the config-2-depth parity tests (tests/test_gpu_deep.py), smoke, a short bench line
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_deep.py > gpurun_out/r5a_deep.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5a_smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 64 --warmup 8 --no-cpu-baseline > gpurun_out/r5a_bench.log 2>&1 || exit $?
