#!/bin/bash
# SQ / TCP / TCC counter passes on the trace kernel of one config (diagnosis, not the bench).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
CFG="${CFG:-C2}"
BENCH="$R/bench.py --config $CFG --no-cpu-baseline --extra= --steps 10 --warmup 1"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" \
           "GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex k_trace_frame -d "$R/gpurun_out/pmc_${CFG}_$i" -o run \
    --output-format csv -- python3 $BENCH > "$R/gpurun_out/pmc_${CFG}_$i.log" 2>&1 || echo "pass $i failed rc=$?"
done
exit 0
