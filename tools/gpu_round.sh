#!/bin/bash
# One GPU-box session: parity tests -> smoke -> bench. Stops at the first GPU fault / abort /
# timeout (exit codes other than 0 and pytest's 1 = "tests failed").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS="${STEPS:-tests bench}"
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
if [[ " $STEPS " == *" tests "* ]]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -rf --timeout=300 ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
  ok $rc || exit $rc
fi
if [[ " $STEPS " == *" smoke "* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
  [ $rc -eq 0 ] || exit $rc
fi
if [[ " $STEPS " == *" bench "* ]]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
