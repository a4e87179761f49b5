#!/bin/bash
# the trace library under two other machine schedulers (-amdgpu-sched-strategy max-ilp / max-memory-clause) against
# the tree's build: frames bit-equal (tools/ab.py), then separate-process timing (tools/lib_ab.py)
set -o pipefail
L=realtimeraytracing_gradproject_amd/lib
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/ab.py --configs C2,C2F,C4,REF,REFL --rounds 2 --steps 10 base=$L/librtamd.so milp=$L/variants/milp/librtamd.so mmc=$L/variants/mmc/librtamd.so > gpurun_out/sched_ab.txt 2>&1 &&
timeout -k 10 840 python3 -u tools/lib_ab.py --roots ab/milp,ab/mmc,. --configs C2,C3,C4,REF,C2F --rounds 4 > gpurun_out/sched_libab.txt 2>&1
