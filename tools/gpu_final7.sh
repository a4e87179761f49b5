#!/bin/bash
# final library: one stress seed, then the share ceilings of C2 and C4
set -o pipefail
STEPS="stress" STRESS_SEED=15 STRESS_MIN=6 TAG=r06s2 bash tools/gpu_r06.sh && \
  STEPS="shares" SHARE_ARGS="--configs C2,C4" TAG=r06s2 bash tools/gpu_r06.sh
