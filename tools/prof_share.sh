#!/bin/bash
# Kernel trace of tools/balance_ab.py on one config / share (run on the GPU box from the repo root): the per-launch
# durations and the gaps between launches of the one-stream loop, balance off (b0) and on (b1).
#   CFG=C4 SHARE=4 bash tools/prof_share.sh   -> gpurun_out/prof_share_<CFG>_n<SHARE>/
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
CFG="${CFG:-C4}"; SHARE="${SHARE:-4}"
O="$R/gpurun_out/prof_share_${CFG}_n${SHARE}"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$O" -o run --output-format csv \
  -- python3 "$R/tools/balance_ab.py" --configs "$CFG" --shares "$SHARE" --rounds 1 --variants b0,b1 \
  > "$O/log.txt" 2>&1 || { echo "prof_share failed rc=$?"; tail -20 "$O/log.txt"; exit 1; }
tail -2 "$O/log.txt"
