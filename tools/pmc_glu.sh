#!/bin/bash
# PMC passes (one counter group per pass) over one decode mat-vec case; usage: tools/pmc_glu.sh CASE OUTDIR [env...]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
case=$1; out=$2; shift 2; mkdir -p $out
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum FETCH_SIZE"; do
  i=$((i+1))
  env "$@" PROBE_CASE="$case" timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o pmc -- python tools/stream_probe.py dec > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $out/p$i.log; }
done
