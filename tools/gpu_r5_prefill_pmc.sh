#!/bin/bash
# prefill PMC passes (tools/pmc_prefill.sh), summarised on the box; only the summary and the logs come back
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
O=/tmp/pmc_r05_prefill
bash tools/pmc_prefill.sh $O > gpurun_out/pmc_r05_prefill.log 2>&1
rc=$?
python3 tools/pmc_prefill_summary.py $O --json gpurun_out/r05_prefill_pmc.json > gpurun_out/pmc_r05_prefill_summary.txt 2>&1
cp $O/p*.log gpurun_out/ 2>/dev/null
exit $rc
