#!/bin/bash
# Round 3 final GPU pass on the final library: -m gpu tests, the default bench line, then the rocprofv3 passes of
# C2 / C4 / C5 (tools/profile_round.sh). Each step under its own limit; stops at the first failure.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
SKIP_TRACE=1 TAG=r03f bash tools/gpu_session.sh || exit 1
TAG=r03 CFGS="${CFGS:-C2 C4 C5}" bash tools/profile_round.sh || exit 1
echo final-ok
