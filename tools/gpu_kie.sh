#!/bin/bash
# key_if_entered in C (RT_KIE_C: s_bfe + v_bfi, no inline-asm hazard nops) against the tree's build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u tools/lib_ab.py --roots ab/kie,. --configs C2,C3,C4,REF,C2F --rounds 5 > gpurun_out/kie_libab.txt 2>&1
