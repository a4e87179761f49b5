#!/bin/bash
# final library, part 3: share ceilings (C2, C4), the strips loop's kernels at C2 N = 8 under a kernel trace, and
# one stress seed
set -o pipefail
R=$(pwd)
STEPS="shares" SHARE_ARGS="--configs C2,C4" TAG=r06v bash tools/gpu_r06.sh && {
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/asm_trace_v" -o run --output-format csv \
    -- python3 "$R/tools/share_ceiling.py" --configs C2 --ranks 8 > "$R/gpurun_out/asm_trace_v.log" 2>&1; } && {
  cd "$R"; STEPS="stress" STRESS_SEED=14 STRESS_MIN=6 TAG=r06v bash tools/gpu_r06.sh; }
