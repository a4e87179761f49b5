#!/bin/bash
# Counter passes on the trace kernel of a given library build (LIB=path CFG=name TAG=label).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
CFG="${CFG:-C2}"; TAG="${TAG:-x}"; LIB="${LIB:-realtimeraytracing_gradproject_amd/lib/librtamd.so}"
case "$LIB" in /*) ;; *) LIB="$R/$LIB" ;; esac
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" \
           "GRBM_GUI_ACTIVE SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex k_trace_frame -d "$R/gpurun_out/pmc_${TAG}_${CFG}_$i" -o run \
    --output-format csv -- python3 "$R/tools/one_config.py" --lib "$LIB" --config "$CFG" > "$R/gpurun_out/pmc_${TAG}_${CFG}_$i.log" 2>&1 || echo "pass $i failed rc=$?"
done
exit 0
