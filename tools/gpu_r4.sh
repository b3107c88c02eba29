#!/bin/bash
# round-4 GPU session: the prefill GEMM A/B (v4 / v5, with and without SLP-packed f32), the whole GPU suite, the
# bench A/B of non-temporal K/V loads in decode attention, and the engine variants + stamps.  Logs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for lib in koboldcpp_hipblas koboldcpp_hipblas_noslp; do
  [ -f koboldcpp_amd/$lib.so ] || continue
  KCPP_LIB=$PWD/koboldcpp_amd/$lib.so timeout -k 10 240 python -u tools/gemm_ab.py 0 14 > gpurun_out/gemm_ab_$lib.log 2>&1 || exit $?
  sed "s/^/$lib /" gpurun_out/gemm_ab_$lib.log
done
GPU_TEST_TIMEOUT=700 bash tools/gpu_tests.sh tests/
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for nt in 0 1; do
  KCPP_FA_NT=$nt timeout -k 10 300 python -u bench.py --steps 64 --warmup 8 --no-cpu-baseline > gpurun_out/bench_nt$nt.log 2>&1 || exit $?
  grep -o '"value": [0-9.]*' gpurun_out/bench_nt$nt.log | head -1 | sed "s/^/fa_nt $nt /"
done
ENG_OPTS="0 170" STAMP_OPT=170 bash tools/gpu_engine_dbg.sh
