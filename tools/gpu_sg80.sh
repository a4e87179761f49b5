#!/bin/bash
# the packet kernels capped at 80 SGPRs (RT_PACKET_SGPRS=80: 72 used, 8 waves per SIMD) against the tree's build
set -o pipefail
L=realtimeraytracing_gradproject_amd/lib
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/ab.py --configs C2,C2F,C4,REF,REFL --rounds 2 --steps 10 base=$L/librtamd.so sg80=$L/variants/sg80/librtamd.so > gpurun_out/sg80_ab.txt 2>&1 &&
timeout -k 10 700 python3 -u tools/lib_ab.py --roots ab/sg80,. --configs C2,C3,C4,REF,C2F,C5 --rounds 4 > gpurun_out/sg80_libab.txt 2>&1
