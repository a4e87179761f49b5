#!/bin/bash
# Counter passes on the raster tile kernel (CFG=config).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
CFG="${CFG:-REF}"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set --kernel-include-regex k_raster -d "$R/gpurun_out/pmcr_${CFG}_$i" -o run \
    --output-format csv -- python3 "$R/tools/raster_prof.py" --config "$CFG" --steps 3 > "$R/gpurun_out/pmcr_${CFG}_$i.log" 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
exit 0
