#!/bin/bash
# final library, part 1: the -m gpu suite, then kernel stats + PMC of C2, C2F, C3, C4
set -o pipefail
STEPS="tests" TAG=r06t bash tools/gpu_r06.sh && CFGS="${PROF_CFGS:-C2 C2F C3 C4}" TAG=r06 bash tools/profile_round.sh
