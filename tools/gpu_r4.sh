#!/bin/bash
# round-4 GPU session: the whole GPU suite, the bench A/B of non-temporal K/V loads in decode attention, and the
# engine variants + stamps.  Logs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
GPU_TEST_TIMEOUT=700 bash tools/gpu_tests.sh tests/
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for nt in 0 1; do
  KCPP_FA_NT=$nt timeout -k 10 300 python -u bench.py --steps 64 --warmup 8 --no-cpu-baseline > gpurun_out/bench_nt$nt.log 2>&1 || exit $?
  grep -o '"value": [0-9.]*' gpurun_out/bench_nt$nt.log | head -1 | sed "s/^/fa_nt $nt /"
done
ENG_OPTS="0 170" STAMP_OPT=170 bash tools/gpu_engine_dbg.sh
