#!/bin/bash
# round-6 final library: rocprofv3 kernel stats + PMC passes of every config (tools/profile_round.sh)
set -o pipefail
CFGS="${PROF_CFGS:-C2 C2F C3 C4 C5 REF C1}" TAG=r06 bash tools/profile_round.sh
