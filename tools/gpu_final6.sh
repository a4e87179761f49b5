#!/bin/bash
# final library, part 2: kernel stats + PMC of the tile-balance configs, then the bench line and the strips lines
set -o pipefail
CFGS="${PROF_CFGS:-C2F C4}" TAG=r06 bash tools/profile_round.sh && \
  STEPS="bench strips5" TAG=r06z STRIPS_CFGS="C2:8 C4:4 C5:8" STRIPS_STEPS=40 bash tools/gpu_r06.sh
