#!/bin/bash
# GPU-box step: parity tests of the current build, then an interleaved A/B of library variants.
#   AB="base=<lib> new=<lib>" CONFIGS=C2,C3 bash tools/gpu_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python -u tools/ab.py --configs "${CONFIGS:-C2,C2F,C3,C4,C5}" --rounds "${ROUNDS:-5}" --steps "${STEPS:-20}" $AB \
  > gpurun_out/ab.log 2>&1
rc=$?; echo "ab rc=$rc"; tail -30 gpurun_out/ab.log
exit $rc
