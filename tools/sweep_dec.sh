#!/bin/bash
# sweep decode launch parameters under rocprofv3; one summary per config (args: list of "blocks R0 R1")
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cfg in "$@"; do
  set -- $cfg
  d=gpurun_out/sweep_$1_$2_$3
  mkdir -p $d
  KCPP_DEC_BLOCKS=$1 KCPP_R0=$2 KCPP_R1=$3 timeout -k 10 120 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python tools/profile_decode.py decode > $d/log 2>&1 || exit 1
  echo "== blocks=$1 R0=$2 R1=$3"; python tools/trace_summary.py $d/run_kernel_trace.csv
done
