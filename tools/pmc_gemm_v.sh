#!/bin/bash
# PMC passes (one block group each) over one prefill GEMM shape and variant (tools/gemm_ab.py)
# usage: tools/pmc_gemm_v.sh OUTDIR SHAPE VARIANT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=$1; shape=$2; v=$3; mkdir -p $out
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
           "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TCP_UTCL1_TRANSLATION_MISS_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" \
           "TD_TD_BUSY_sum TD_TC_STALL_sum SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  GEMM_ONLY="$shape" timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o pmc -- python3 tools/gemm_ab.py $v > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $out/p$i.log; exit 1; }
done
