#!/bin/bash
# Mixtral (BASELINE config 5) with the grouped MoE prefill: kernel-trace stats (stats csv only copied back)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_mix -o mix -- python3 bench.py --config mixtral-8x7b-q5_k_m --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/mixprof.log 2>&1 || exit $?
find /tmp/prof_mix -name "*kernel_stats.csv" -exec cp {} gpurun_out/mixprof_kernel_stats.csv \;
