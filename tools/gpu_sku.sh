#!/bin/bash
# the trace library compiled with -structurizecfg-skip-uniform-regions (uniform branches not structurized) against the
# tree's build: frames bit-equal on every config (tools/ab.py), then separate-process timing (tools/lib_ab.py)
set -o pipefail
L=realtimeraytracing_gradproject_amd/lib
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/ab.py --configs C1,C2,C2F,C3,C4,REF,REFL,REFLO,DEGEN --rounds 3 --steps 10 base=$L/librtamd.so sku=$L/variants/sku/librtamd.so > gpurun_out/sku_ab.txt 2>&1 &&
timeout -k 10 200 python3 -u tools/ab.py --configs C5 --rounds 2 --steps 3 base=$L/librtamd.so sku=$L/variants/sku/librtamd.so >> gpurun_out/sku_ab.txt 2>&1 &&
timeout -k 10 600 python3 -u tools/lib_ab.py --roots ab/sku,. --configs C2,C3,C4,REF,C2F --rounds 5 > gpurun_out/sku_libab.txt 2>&1 &&
# the strips loop's assembly and gather copy at C2 N = 8 (rank 0's share) under a kernel trace
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OLDPWD/gpurun_out/asm_trace" -o run --output-format csv \
  -- python3 "$OLDPWD/tools/share_ceiling.py" --configs C2 --ranks 8 > "$OLDPWD/gpurun_out/asm_trace.log" 2>&1
