#!/bin/bash
# rocprofv3 passes over the headline bench (run on the GPU box from the repo root):
#   1. kernel trace + stats      -> gpurun_out/prof_kt/
#   2. PMC FETCH_SIZE            -> gpurun_out/prof_fetch/   (TCC counters: FETCH and WRITE need
#   3. PMC WRITE_SIZE            -> gpurun_out/prof_write/    separate passes on gfx950)
# then tools/pmc_summary.py condenses them into profiles/.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r01}"
CFG="${CFG:-C2}"
BENCH="$R/bench.py --config $CFG --no-cpu-baseline --extra="
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_kt" -o run --output-format csv \
  -- python3 $BENCH --steps 200 --warmup 100 > "$R/gpurun_out/prof_kt.log" 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_trace_frame -d "$R/gpurun_out/prof_fetch" \
  -o run --output-format csv -- python3 $BENCH --steps 20 --warmup 100 > "$R/gpurun_out/prof_fetch.log" 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_trace_frame -d "$R/gpurun_out/prof_write" \
  -o run --output-format csv -- python3 $BENCH --steps 20 --warmup 100 > "$R/gpurun_out/prof_write.log" 2>&1 || exit $?
echo "profiles: run python3 tools/pmc_summary.py --tag $TAG --config $CFG locally after the merge"
