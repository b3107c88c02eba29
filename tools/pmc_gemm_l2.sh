#!/bin/bash
# L2 hit/miss and HBM fetch of the prefill GEMM at one shape (tools/gemm_ab.py), one counter group per pass
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=$1; shape=$2; mkdir -p $out
i=0
for grp in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" "TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  GEMM_ONLY="$shape" timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o pmc -- python3 tools/gemm_ab.py 3 > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $out/p$i.log; exit 1; }
done
