#!/bin/bash
# engine diagnostics on the GPU box: bitwise engine tests, the bench with the engine at several edge orderings
# (KCPP_ENGINE_OPT), then the phase timeline
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_gpu_engine.py > gpurun_out/eng_dbg.log 2>&1
rc=$?
echo "rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for o in ${ENG_OPTS:-0}; do
  KCPP_ENGINE_OPT=$o timeout -k 10 300 python -u bench.py --steps 64 --warmup 8 --no-cpu-baseline --engine 1 > gpurun_out/eng_bench_$o.log 2>&1 || exit $?
  grep -o '"value": [0-9.]*' gpurun_out/eng_bench_$o.log | head -1 | sed "s/^/opt $o /"
done
KCPP_ENGINE_OPT=${STAMP_OPT:-0} timeout -k 10 200 python -u tools/engine_stamps.py > gpurun_out/eng_stamps.log 2>&1 || exit $?
