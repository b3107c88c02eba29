#!/bin/bash
# Round profile: the PMC passes and kernel-trace stats that back bench.py's `roofline` object, plus a
# kernel-trace of a short full bench.  Usage (on the GPU box): tools/profile_round.sh TAG
# Writes gpurun_out/prof_TAG/...; tools/roofline_summary.py then writes profiles/TAG_*.
set -o pipefail
TAG=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
# 1/2: memory-side bytes of the dominant decode kernel, one counter per pass (FETCH_SIZE and WRITE_SIZE
# cannot share a pass on gfx950), no tracing domains combined with --pmc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o roof -- python3 bench.py --roofline-only > $OUT/fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o roof -- python3 bench.py --roofline-only > $OUT/write.log 2>&1 &&
# 3: kernel-trace stats of the same command (average launch duration must agree with bench's HIP events)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o roof -- python3 bench.py --roofline-only > $OUT/trace.log 2>&1 &&
# 5/6: memory-side bytes of the decode attention (k_fa_dec4 + k_fa_comb4 at 3850 cached keys, 32 layers' caches
# rotated past the Infinity Cache), one counter per pass, and its kernel-trace stats
FA_VARIANTS=3 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fa_fetch -o fa -- python3 tools/fa_dec_bench.py 3850 > $OUT/fa_fetch.log 2>&1 &&
FA_VARIANTS=3 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/fa_write -o fa -- python3 tools/fa_dec_bench.py 3850 > $OUT/fa_write.log 2>&1 &&
FA_VARIANTS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/fa_trace -o fa -- python3 tools/fa_dec_bench.py 3850 > $OUT/fa_trace.log 2>&1 &&
# 4: kernel-trace stats of a short full bench (prefill + decode), no CPU baseline
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench -o bench -- python3 bench.py --steps 32 --warmup 4 --no-cpu-baseline > $OUT/bench.log 2>&1
rc=$?
echo "profile_round rc=$rc"
exit $rc
