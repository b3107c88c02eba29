#!/bin/bash
# Prefill MFMA-utilisation passes over the bench workload (Llama-3-8B Q4_K_M, 3840-token prompt in 512-token
# ubatches): one counter group per rocprofv3 --pmc pass (never combined with tracing), then a kernel trace.
# usage: tools/pmc_prefill.sh OUTDIR        summary: python tools/pmc_prefill_summary.py OUTDIR
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=$1; mkdir -p $out
B="bench.py --no-cpu-baseline --steps 2 --warmup 1"
timeout -k 10 120 rocprofv3 --list-avail > $out/avail.txt 2>&1 || true
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES" \
           "$PMC_EXTRA"; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  keep=""; for c in $grp; do grep -q "\b$c\b" $out/avail.txt && keep="$keep $c" || echo "skip $c (not listed)"; done
  grp=$keep
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o pmc -- python3 $B > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $out/p$i.log; exit 1; }
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o tr -- python3 $B > $out/trace.log 2>&1
