#!/bin/bash
# One GPU call of a working session (run on the GPU box from the repo root): the -m gpu tests, the default
# bench line, and the frames-in-flight kernel trace. Each step under its own time limit; the
# script stops at the first failure.
#   TAG=r03a bash tools/gpu_session.sh
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r03}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$O/gputest_${TAG}.log" 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 "$O/gputest_${TAG}.log"; exit 1; }
  tail -3 "$O/gputest_${TAG}.log"
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 600 python3 bench.py > "$O/bench_${TAG}.json" 2> "$O/bench_${TAG}.err" \
    || { echo "bench failed rc=$?"; tail -20 "$O/bench_${TAG}.err"; exit 1; }
  echo "bench ok"
fi
if [ "${SKIP_TRACE:-0}" != "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_${TAG}_C2_if3" -o run --output-format csv \
    -- python3 "$R/bench.py" --config C2 --no-cpu-baseline --extra= --steps 200 --warmup 100 --in-flight 3 \
    > "$O/prof_${TAG}_C2_if3.log" 2>&1 || { echo "in-flight trace failed rc=$?"; exit 1; }
  echo "trace ok"
fi
exit 0
