#!/bin/bash
# Host sanitizer check, CPU only, CI-style: builds the ASan + UBSan variants of the
# product library's host C++ and of the oracle (make asan), runs the standalone ingest / manipulator fuzz driver, then
# the CPU tests of the ingest (incl. the malformed-OBJ cases pinned to the reference's loader), the manipulator and
# the oracle with python loading the sanitized libraries (RT_LIBRARY / ORACLE_LIBRARY, gcc's runtimes preloaded).
# Any sanitizer report aborts (halt_on_error) and the script exits non-zero.
#   bash tools/asan_check.sh            (from the repo root; ~2 min)
set -euo pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"
make -j8 realtimeraytracing_gradproject_amd/lib/librtamd.so > /dev/null
make asan > /dev/null
export ASAN_OPTIONS=detect_leaks=0:detect_odr_violation=0:alloc_dealloc_mismatch=0:halt_on_error=1:abort_on_error=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
./build/asan/obj_ingest_fuzz 20000
PRE="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)"
export RT_LIBRARY="$R/build/asan/librtamd.so" ORACLE_LIBRARY="$R/build/asan/liboracle.so"
# the sanitized libraries are the ones loaded, and the sanitizer runtime is in the process
LD_PRELOAD="$PRE" python3 - <<'PY'
import realtimeraytracing_gradproject_amd as rt, oracle
maps = open("/proc/self/maps").read()
assert rt.LIB_PATH.endswith("build/asan/librtamd.so") and oracle.LIB_PATH.endswith("build/asan/liboracle.so")
assert "libasan.so" in maps and "build/asan/librtamd.so" in maps and "build/asan/liboracle.so" in maps
print("sanitized libraries loaded:", rt.LIB_PATH, oracle.LIB_PATH)
PY
LD_PRELOAD="$PRE" timeout 1800 python3 -m pytest -q -p no:cacheprovider -m "not gpu" \
  tests/test_ingest.py tests/test_manipulator.py tests/test_camera.py tests/test_oracle.py
echo "asan_check: clean"
