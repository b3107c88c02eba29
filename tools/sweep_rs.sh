#!/bin/bash
# RS decode mat-vec launch sweep (tools only): one probe process per (R, PF, blocks) setting
cd "$GRAFT_REPO_ROOT" || exit 1
for cfg in "$@"; do
  set -- $cfg
  KCPP_RS_R=$1 KCPP_RS_PF=$2 KCPP_RS_BLOCKS=$3 PROBE_RS_ONLY=1 timeout -k 10 100 python3 tools/stream_probe.py dec 2>/dev/null \
    | sed "s/^/R=$1 PF=$2 B=$3 /" || exit 1
done
