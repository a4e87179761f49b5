#!/bin/bash
# One GPU call of a round-6 session (run on the GPU box from the repo root). STEPS selects: tests, bench, strips5,
# shares, balance, waves. Each step under its own time limit; the script stops at the first failure.
#   STEPS="tests bench" TAG=r06a bash tools/gpu_r06.sh
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r06}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
for step in ${STEPS:-tests}; do
  case $step in
    tests)
      timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v ${PYTEST_EXTRA:-} --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
        > "$O/gputest_${TAG}.log" 2>&1 || { echo "gpu tests failed rc=$?"; grep -E "FAIL|Error|error" "$O/gputest_${TAG}.log" | head -20; tail -40 "$O/gputest_${TAG}.log"; exit 1; }
      tail -3 "$O/gputest_${TAG}.log" ;;
    bench)
      timeout -k 10 600 python3 bench.py ${BENCH_ARGS:-} > "$O/bench_${TAG}.json" 2> "$O/bench_${TAG}.err" \
        || { echo "bench failed rc=$?"; tail -20 "$O/bench_${TAG}.err"; exit 1; }
      head -c 1500 "$O/bench_${TAG}.json"; echo ;;
    strips5)
      # the C5 (4 spp, 4K) and C4 tiled loops through the loopback transport
      for cfg in ${STRIPS_CFGS:-C5:8 C4:4}; do
        set -- ${cfg%%:*} ${cfg#*:}
        timeout -k 10 300 python3 bench.py --mode strips --loopback $2 --config $1 --extra= --no-cpu-baseline \
          --steps ${STRIPS_STEPS:-40} --warmup 8 \
          > "$O/strips_${1}_lb${2}_${TAG}.json" 2> "$O/strips_${1}_lb${2}_${TAG}.err" \
          || { echo "strips loopback $1 $2 failed rc=$?"; tail -20 "$O/strips_${1}_lb${2}_${TAG}.err"; exit 1; }
        head -c 900 "$O/strips_${1}_lb${2}_${TAG}.json"; echo
      done ;;
    shares)
      timeout -k 10 900 python3 -u tools/share_ceiling.py ${SHARE_ARGS:-} > "$O/shares_${TAG}.jsonl" 2> "$O/shares_${TAG}.err" \
        || { echo "share_ceiling failed rc=$?"; tail -20 "$O/shares_${TAG}.err"; exit 1; }
      cat "$O/shares_${TAG}.jsonl" ;;
    libab)
      timeout -k 10 900 python3 tools/lib_ab.py --roots ${AB_ROOTS:-ab/r03,.,.:bal0} --configs ${AB_CONFIGS:-C2,C2F,C4} \
        --rounds ${AB_ROUNDS:-5} > "$O/libab_${TAG}.txt" 2>&1 || { echo "lib_ab failed rc=$?"; tail -20 "$O/libab_${TAG}.txt"; exit 1; }
      tail -40 "$O/libab_${TAG}.txt" ;;
    prof)
      CFGS="${PROF_CFGS:-C2 C4 C5}" TAG="$TAG" bash tools/profile_round.sh || { echo "profile_round failed"; exit 1; } ;;
    sqc)
      # scalar data cache hit rate of the trace kernel (one pass; counters of the SQC block only)
      cd /tmp && export TMPDIR=/tmp
      timeout -s KILL 90 rocprofv3 --pmc ${SQC_SET:-SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE} \
        --kernel-include-regex k_trace_frame -d "$O/sqc_${TAG}" -o run --output-format csv \
        -- python3 "$R/tools/one_config.py" --config ${SQC_CONFIG:-C2} --frames 12 > "$O/sqc_${TAG}.log" 2>&1 \
        || { echo "sqc pass failed rc=$?"; tail -20 "$O/sqc_${TAG}.log"; exit 1; }
      cd "$R"; find "$O/sqc_${TAG}" -name "*counter_collection.csv" | head -1 | xargs -r tail -5 ;;
    clock)
      # do the recording kernel's clock reads fetch from the fabric? (tools/clock_probe.hip)
      cd /tmp && export TMPDIR=/tmp
      for ctr in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 60 rocprofv3 --pmc $ctr --kernel-include-regex k_clock -d "$O/clock_${TAG}_$ctr" -o run \
          --output-format csv -- "$R/tools/bin/clock_probe" > "$O/clock_${TAG}_$ctr.log" 2>&1 \
          || { echo "clock probe $ctr failed rc=$?"; tail -20 "$O/clock_${TAG}_$ctr.log"; exit 1; }
      done
      cd "$R"; find "$O/clock_${TAG}_FETCH_SIZE" -name "*counter_collection.csv" | head -1 | xargs -r cat | head -12 ;;
    planstream)
      # A/B: the plans on the context stream vs a high-priority stream of their own (RT_PLAN_STREAM_PRIO), twice each
      cd /tmp && export TMPDIR=/tmp
      for rep in 1 2; do
        for ps in 0 1; do
          export RT_PLAN_STREAM_PRIO=$ps
          timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/planstream_${TAG}_${ps}_$rep" -o run --output-format csv \
            -- python3 "$R/tools/plan_load.py" --configs C2F,C4,C4/4,C2@3,C4@3 --frames 400 > "$O/planstream_${TAG}_${ps}_$rep.log" 2>&1 \
            || { echo "planstream $ps failed rc=$?"; tail -20 "$O/planstream_${TAG}_${ps}_$rep.log"; exit 1; }
          unset RT_PLAN_STREAM_PRIO
          echo "== plan stream prio $ps rep $rep"; grep '^{' "$O/planstream_${TAG}_${ps}_$rep.log"
          find "$O/planstream_${TAG}_${ps}_$rep" -name "*kernel_stats.csv" | head -1 | xargs -r grep -E "k_tile_plan" | cut -c1-160
        done
      done
      cd "$R" ;;
    planload)
      # k_tile_plan under load, per library build (PLAN_LIBS), rocprofv3 kernel stats of each
      cd /tmp && export TMPDIR=/tmp
      for lib in ${PLAN_LIBS:-realtimeraytracing_gradproject_amd/lib/librtamd.so}; do
        nm=$(basename $(dirname $lib))
        timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/planload_${TAG}_$nm" -o run --output-format csv \
          -- python3 "$R/tools/plan_load.py" --lib "$R/$lib" > "$O/planload_${TAG}_$nm.log" 2>&1 \
          || { echo "plan_load $nm failed rc=$?"; tail -20 "$O/planload_${TAG}_$nm.log"; exit 1; }
        grep '^{' "$O/planload_${TAG}_$nm.log"
        find "$O/planload_${TAG}_$nm" -name "*kernel_stats.csv" | head -1 | xargs -r grep -E "k_tile_plan|Name" | cut -c1-200
      done
      cd "$R" ;;
    fetchab)
      # where the recording kernel's extra HBM reads come from — FETCH_SIZE per dispatch of C2F / C4
      # with the balance off, adaptive, adaptive without splits or front class (the list never pays: the plain
      # kernel, recording on some launches), and the forced 4-part layout (a plan before every launch)
      cd /tmp && export TMPDIR=/tmp
      for cfg in ${FAB_CFGS:-C2F C4}; do
        for v in ${FAB_SET:-off:--balance=0 adaptive: recordonly: listonly: forced4:--balance=2}; do
          nm=${v%%:*}; args=${v#*:}
          unset RT_BALANCE_SPLIT RT_BALANCE_FRONT RT_BALANCE_DIAG
          if [ "$nm" = nosplit ]; then export RT_BALANCE_SPLIT=0 RT_BALANCE_FRONT=0; fi
          if [ "$nm" = recordonly ]; then export RT_BALANCE_DIAG=1; fi
          if [ "$nm" = listonly ]; then export RT_BALANCE_DIAG=2; fi
          if [ "$nm" = plainlist ]; then export RT_BALANCE_DIAG=3 RT_BALANCE_SPLIT=0 RT_BALANCE_FRONT=0; fi
          if [ "$nm" = frontlist ]; then export RT_BALANCE_DIAG=3 RT_BALANCE_SPLIT=0; fi
          if [ "$nm" = splitlist ]; then export RT_BALANCE_DIAG=3 RT_BALANCE_FRONT=0; fi
          timeout -s KILL 90 rocprofv3 --pmc ${FAB_CTR:-FETCH_SIZE} -d "$O/fab_${TAG}_${cfg}_$nm" -o run \
            --output-format csv -- python3 "$R/tools/one_config.py" --config $cfg --frames 24 $args \
            > "$O/fab_${TAG}_${cfg}_$nm.log" 2>&1 || { echo "fetchab $cfg $nm failed rc=$?"; tail -5 "$O/fab_${TAG}_${cfg}_$nm.log"; exit 1; }
          unset RT_BALANCE_SPLIT RT_BALANCE_FRONT RT_BALANCE_DIAG
          echo "== $cfg $nm"
          find "$O/fab_${TAG}_${cfg}_$nm" -name "*counter_collection.csv" | head -1 | xargs -r \
            python3 -c "import csv,sys; [print(r['Dispatch_Id'], r['Kernel_Name'][:70], r['Counter_Value']) for r in csv.DictReader(open(sys.argv[1]))]" | tail -14
        done
      done
      cd "$R" ;;
    stress)
      # one long seed per kernel change
      timeout -k 10 900 python3 -u tools/stress.py --minutes ${STRESS_MIN:-8} --seed ${STRESS_SEED:-12} \
        > "$O/stress_${TAG}.log" 2>&1 || { echo "stress failed rc=$?"; tail -30 "$O/stress_${TAG}.log"; exit 1; }
      tail -3 "$O/stress_${TAG}.log" ;;
    queue)
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$O/queue_${TAG}" -o run --output-format csv \
        -- python3 "$R/tools/queue_probe.py" > "$O/queue_${TAG}.log" 2>&1 \
        || { echo "queue probe failed rc=$?"; tail -20 "$O/queue_${TAG}.log"; exit 1; }
      cd "$R"; find "$O/queue_${TAG}" -name "*kernel_trace.csv" | head -1 | xargs -r python3 tools/queue_summary.py ;;
    occ)
      timeout -k 10 120 ./tools/bin/occupancy_probe > "$O/occupancy_${TAG}.jsonl" 2>&1 \
        || { echo "occupancy_probe failed rc=$?"; tail -20 "$O/occupancy_${TAG}.jsonl"; exit 1; }
      cat "$O/occupancy_${TAG}.jsonl" ;;
    ab)
      # one-process interleaved A/B of library variants (tools/ab.py; AB_VARIANTS name=lib ...)
      timeout -k 10 900 python3 tools/ab.py ${AB_ARGS:-} ${AB_VARIANTS} > "$O/ab_${TAG}.txt" 2>&1 \
        || { echo "ab failed rc=$?"; tail -20 "$O/ab_${TAG}.txt"; exit 1; }
      tail -40 "$O/ab_${TAG}.txt" ;;
    balance)
      timeout -k 10 600 python3 tools/balance_ab.py ${BAL_ARGS:-} > "$O/balance_${TAG}.txt" 2>&1 \
        || { echo "balance_ab failed rc=$?"; tail -20 "$O/balance_${TAG}.txt"; exit 1; }
      cat "$O/balance_${TAG}.txt" ;;
    waves)
      for b in ${WT_BAL:-0 1}; do
        timeout -k 10 120 python3 tools/wave_times.py --lib ${WT_LIB:-realtimeraytracing_gradproject_amd/lib/variants/wavetimes/librtamd.so} \
          --config ${WT_CONFIG:-C4} --balance $b ${WT_ARGS:-} > "$O/wave_times_${TAG}_b$b.txt" 2>&1 \
          || { echo "wave_times failed rc=$?"; tail -20 "$O/wave_times_${TAG}_b$b.txt"; exit 1; }
        cat "$O/wave_times_${TAG}_b$b.txt"
      done ;;
  esac
done
exit 0
