#!/bin/bash
# Mixtral (BASELINE config 5): bench line + kernel-trace stats
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --config mixtral-8x7b-q5_k_m > gpurun_out/r5_mix.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r5_mix -o mix -- python3 bench.py --config mixtral-8x7b-q5_k_m --steps 32 --warmup 4 --no-cpu-baseline > gpurun_out/r5_mix_prof.log 2>&1 || exit $?
