#!/bin/bash
# BLAS push / pop write skips (RT_PUSH_SKIP / RT_POP_SKIP) against the tree's build, separate processes; then the
# -m gpu suite on the tree's build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python3 -u tools/lib_ab.py --roots ab/push,ab/pop,ab/pp,. --configs C2,C3,C4,REF --rounds 4 > gpurun_out/pp_libab.txt 2>&1 &&
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_r06n.log 2>&1
rc=$?; tail -3 gpurun_out/gputest_r06n.log; exit $rc
