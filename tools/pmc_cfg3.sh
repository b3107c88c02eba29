#!/bin/bash
# BASELINE config 3 profile (round 5): kernel-trace stats of the config-3 bench, and per GEMM shape (tools/q80t_shapes.py)
# FETCH_SIZE / WRITE_SIZE passes (one counter block per pass) plus an SQ pass; summarised by tools/pmc_cfg3_summary.py
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/pmc_cfg3
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o cfg3 -- python3 bench.py --config llama3-8b-q8_0-b32 --steps 8 --warmup 2 --no-cpu-baseline > $O/trace.log 2>&1 || exit $?
for sh in qkv wo down gate_up; do
  timeout -k 10 120 python3 tools/q80t_shapes.py $sh > $O/time_$sh.json 2> $O/time_$sh.err || exit $?
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$sh -o p -- python3 tools/q80t_shapes.py $sh > $O/fetch_$sh.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$sh -o p -- python3 tools/q80t_shapes.py $sh > $O/write_$sh.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d $O/sq_$sh -o p -- python3 tools/q80t_shapes.py $sh > $O/sq_$sh.log 2>&1 || exit $?
done
echo pmc_cfg3 done
