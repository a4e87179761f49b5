#!/bin/bash
# one GPU call for several experiment scripts, each ended by its own failure
set -o pipefail
bash tools/gpu_cand.sh && TAG=hwq bash tools/gpu_hwq.sh
