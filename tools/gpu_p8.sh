#!/bin/bash
# the 8-wave frame kernel (k_trace_frame_packet8, RT_PLAIN_SGPRS) against the library before it (ab/prev), then the
# -m gpu suite on the tree's build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python3 -u tools/lib_ab.py --roots ab/prev,. --configs C2,C3,C4,REF,C2F,C5 --rounds 4 > gpurun_out/p8_libab.txt 2>&1 &&
STEPS="tests" TAG=r06y bash tools/gpu_r06.sh
