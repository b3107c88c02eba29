#!/bin/bash
# PMC passes over the prefill flash attention (tools/fa_ab.py) at one depth and variant
# usage: tools/pmc_fa.sh OUTDIR NPAST VARIANT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=$1; np=$2; v=$3; mkdir -p $out
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  FA_NPAST=$np timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o pmc -- python3 tools/fa_ab.py $v > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $out/p$i.log; exit 1; }
done
