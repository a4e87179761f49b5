#!/bin/bash
# One GPU call of a round-4 session (run on the GPU box from the repo root). STEPS selects: tests, bench, balance,
# waves, strips. Each step under its own time limit; the script stops at the first failure.
#   STEPS="bench balance" TAG=r04a bash tools/gpu_r04.sh
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r04}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
for step in ${STEPS:-tests}; do
  case $step in
    tests)
      timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
        > "$O/gputest_${TAG}.log" 2>&1 || { echo "gpu tests failed rc=$?"; tail -40 "$O/gputest_${TAG}.log"; exit 1; }
      tail -3 "$O/gputest_${TAG}.log" ;;
    bench)
      timeout -k 10 600 python3 bench.py > "$O/bench_${TAG}.json" 2> "$O/bench_${TAG}.err" \
        || { echo "bench failed rc=$?"; tail -20 "$O/bench_${TAG}.err"; exit 1; }
      head -c 1500 "$O/bench_${TAG}.json"; echo ;;
    balance)
      timeout -k 10 600 python3 tools/balance_ab.py ${BAL_ARGS:-} > "$O/balance_${TAG}.txt" 2>&1 \
        || { echo "balance_ab failed rc=$?"; tail -20 "$O/balance_${TAG}.txt"; exit 1; }
      cat "$O/balance_${TAG}.txt" ;;
    waves)
      for b in 0 1; do
        timeout -k 10 120 python3 tools/wave_times.py --lib realtimeraytracing_gradproject_amd/lib/variants/wavetimes/librtamd.so \
          --config ${WT_CONFIG:-C4} --balance $b ${WT_ARGS:-} > "$O/wave_times_${TAG}_b$b.txt" 2>&1 \
          || { echo "wave_times failed rc=$?"; tail -20 "$O/wave_times_${TAG}_b$b.txt"; exit 1; }
        cat "$O/wave_times_${TAG}_b$b.txt"
      done ;;
    strips)
      for n in 2 4 8; do
        timeout -k 10 300 python3 bench.py --mode strips --loopback $n --extra= --no-cpu-baseline --steps 200 --warmup 50 \
          > "$O/strips_lb${n}_${TAG}.json" 2> "$O/strips_lb${n}_${TAG}.err" \
          || { echo "strips loopback $n failed rc=$?"; tail -20 "$O/strips_lb${n}_${TAG}.err"; exit 1; }
        head -c 900 "$O/strips_lb${n}_${TAG}.json"; echo
      done ;;
  esac
done
exit 0
