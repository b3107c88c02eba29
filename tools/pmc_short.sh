#!/bin/bash
# HBM bytes (FETCH_SIZE / WRITE_SIZE, one counter per pass) and kernel-trace durations of the short decode
# mat-vecs (wo, q|k|v) in the stream probe (weights rotated past the Infinity Cache); usage (GPU box):
#   tools/pmc_short.sh OUTDIR ; then python tools/pmc_short_summary.py OUTDIR > profiles/<tag>_short_matvec_pmc.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=${1:-gpurun_out/pmc_short}
mkdir -p $out
i=0
for c in "rs wo q4k pro0" "rs qkv q4k pro1 rope" "rs down q4k pro2" "rs down q6k pro2"; do
  i=$((i+1)); mkdir -p $out/c$i
  for ctr in FETCH_SIZE WRITE_SIZE; do
    PROBE_CASE="$c" timeout -k 10 120 rocprofv3 --pmc $ctr --output-format csv -d $out/c$i/$ctr -o pmc -- python3 tools/stream_probe.py dec > $out/c$i/$ctr.log 2>&1 || exit $?
  done
  PROBE_CASE="$c" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c$i/trace -o tr -- python3 tools/stream_probe.py dec > $out/c$i/trace.log 2>&1 || exit $?
  echo "$c" > $out/c$i/case.txt
done
