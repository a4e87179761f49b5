#!/bin/bash
# A/B of the TLAS push trim (RT_TLAS_PUSH_TRIM) against the product build: separate processes (lib_ab), then the
# in-process rank-share A/B
set -o pipefail
L=realtimeraytracing_gradproject_amd/lib
mkdir -p gpurun_out
timeout -k 10 600 python3 -u tools/lib_ab.py --roots ab/tlastrim,. --configs C2,C2F,C3,C4,REF --rounds 5 > gpurun_out/trim_libab.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --configs C4 --share 4 --rounds 15 --steps 40 base=$L/librtamd.so trim=$L/variants/tlastrim/librtamd.so base2=$L/librtamd.so > gpurun_out/trim_share4.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --configs C2F --rounds 15 --steps 40 base=$L/librtamd.so trim=$L/variants/tlastrim/librtamd.so base2=$L/librtamd.so > gpurun_out/trim_c2f.txt 2>&1
