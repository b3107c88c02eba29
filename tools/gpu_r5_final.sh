#!/bin/bash
# round-5 measurement: the default bench line, then the round profile (roofline PMC passes, FA PMC, bench kernel stats)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/r5_bench.log 2>&1 || exit $?
bash tools/profile_round.sh r05 > gpurun_out/r5_profile.log 2>&1 || exit $?
