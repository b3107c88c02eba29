#!/bin/bash
# run the decode profile once per environment setting given as arguments ("VAR=val VAR2=val")
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for cfg in "$@"; do
  i=$((i+1)); d=gpurun_out/sweepenv_$i; mkdir -p $d
  env $cfg timeout -k 10 120 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python tools/profile_decode.py decode > $d/log 2>&1 || exit 1
  echo "== $cfg"; python tools/trace_summary.py $d/run_kernel_trace.csv > $d/summary.txt; head -8 $d/summary.txt; tail -1 $d/summary.txt
done
