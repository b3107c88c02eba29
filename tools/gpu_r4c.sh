#!/bin/bash
# round-4 GPU session C: round profiles (roofline PMC + traces, decode attention, full bench trace), the short
# mat-vec PMC and the prefill PMC passes.  Summaries: tools/roofline_summary.py r04, pmc_short_summary.py,
# pmc_prefill_summary.py.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
bash tools/profile_round.sh r04 || exit $?
bash tools/pmc_prefill.sh gpurun_out/pmc_prefill_r04 || exit $?
bash tools/pmc_short.sh gpurun_out/pmc_short_r04 || exit $?
