#!/bin/bash
# One WRITE_SIZE counter pass (its own rocprofv3 run, TCC slots) over a few frames of CFG with library LIB:
#   LIB=path CFG=C5 TAG=label bash tools/pmc_write.sh  -> gpurun_out/pmcw_<TAG>_<CFG>/
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
CFG="${CFG:-C5}"; TAG="${TAG:-x}"; LIB="${LIB:-realtimeraytracing_gradproject_amd/lib/librtamd.so}"
case "$LIB" in /*) ;; *) LIB="$R/$LIB" ;; esac
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_trace_frame -d "$R/gpurun_out/pmcw_${TAG}_${CFG}" \
  -o run --output-format csv -- python3 "$R/tools/one_config.py" --lib "$LIB" --config "$CFG" --frames 6 \
  > "$R/gpurun_out/pmcw_${TAG}_${CFG}.log" 2>&1
