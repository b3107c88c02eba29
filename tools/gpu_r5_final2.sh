#!/bin/bash
# round-5 close: the whole GPU suite, smoke(), the default bench line, config 3
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/fin_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/fin_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/fin_bench.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config llama3-8b-q8_0-b32 --steps 32 --warmup 4 > gpurun_out/fin_cfg3.log 2>&1 || exit $?
