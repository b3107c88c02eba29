#!/bin/bash
# engine parity vs the launch chain + round-4 tests, then a short bench (engine on, then off)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_rope_config.py tests/test_gpu_expose.py "tests/test_gpu_fullsize.py::test_ubatch_invariance_legacy_types" > gpurun_out/eng_test.log 2>&1
rc=$?
echo "test rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 64 --warmup 8 --no-cpu-baseline > gpurun_out/eng_bench.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 64 --warmup 8 --no-cpu-baseline --no-engine > gpurun_out/eng_bench_off.log 2>&1 || exit $?
exit $rc
