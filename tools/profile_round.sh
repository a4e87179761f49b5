#!/bin/bash
# rocprofv3 passes of a round (run on the GPU box from the repo root), per config:
#   kt    kernel trace + stats over bench.py, one frame in flight (per-launch durations not
#         stretched by a concurrent frame)              -> gpurun_out/prof_<tag>_<cfg>_kt/
#   pmc1  FETCH_SIZE                                   -> gpurun_out/prof_<tag>_<cfg>_pmc1/
#   pmc2  WRITE_SIZE (TCC slots: not with FETCH_SIZE)  -> gpurun_out/prof_<tag>_<cfg>_pmc2/
#   pmc3  wave / issue-stall SQ counters               -> gpurun_out/prof_<tag>_<cfg>_pmc3/
#   pmc4  instruction mix + GRBM_GUI_ACTIVE            -> gpurun_out/prof_<tag>_<cfg>_pmc4/
# Every pass is its own run under its own time limit; the script stops at the first failure.
# Then, locally: python3 tools/roofline.py summarize --tag <tag> --config <cfg>
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r02}"
CFGS="${CFGS:-C2}"
O="$R/gpurun_out"
mkdir -p "$O"
sha256sum "$R/realtimeraytracing_gradproject_amd/lib/librtamd.so" > "$O/prof_${TAG}_libsha.txt"
cd /tmp && export TMPDIR=/tmp
for CFG in $CFGS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_${TAG}_${CFG}_kt" -o run --output-format csv \
    -- python3 "$R/bench.py" --config "$CFG" --no-cpu-baseline --extra= --steps 100 --warmup 20 --in-flight 1 \
    > "$O/prof_${TAG}_${CFG}_kt.log" 2>&1 || { echo "kt $CFG failed rc=$?"; exit 1; }
  i=0
  for set in "FETCH_SIZE" "WRITE_SIZE" \
             "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
             "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex k_trace_frame -d "$O/prof_${TAG}_${CFG}_pmc$i" \
      -o run --output-format csv -- python3 "$R/tools/one_config.py" --config "$CFG" --frames 12 \
      > "$O/prof_${TAG}_${CFG}_pmc$i.log" 2>&1 || { echo "pmc$i $CFG failed rc=$?"; exit 1; }
  done
  echo "profiled $CFG"
done
exit 0
