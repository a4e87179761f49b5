#!/bin/bash
# final library (8-wave frame kernel), part 1: kernel stats + PMC of the configs whose kernel changed
set -o pipefail
CFGS="${PROF_CFGS:-C2 C3 C5 REF C1}" TAG=r06 bash tools/profile_round.sh
