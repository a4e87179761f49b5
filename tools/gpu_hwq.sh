#!/bin/bash
# k_tile_plan's loaded duration and the frame loops with more hardware queues per process:
# the plan stream shares one of HIP's 4 default queues with a frame stream; GPU_MAX_HW_QUEUES=8 gives each its own.
set -o pipefail
R=$(pwd); O=$R/gpurun_out; TAG=${TAG:-hwq}; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for q in 4 8; do
  export GPU_MAX_HW_QUEUES=$q
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/planload_${TAG}_q$q" -o run --output-format csv \
    -- python3 "$R/tools/plan_load.py" > "$O/planload_${TAG}_q$q.log" 2>&1 \
    || { echo "plan_load q$q failed rc=$?"; tail -20 "$O/planload_${TAG}_q$q.log"; exit 1; }
  grep '^{' "$O/planload_${TAG}_q$q.log"
  find "$O/planload_${TAG}_q$q" -name "*kernel_stats.csv" | head -1 | xargs -r grep -E "k_tile_plan|Name" | cut -c1-200
done
cd "$R"
for q in 4 8 4 8; do
  export GPU_MAX_HW_QUEUES=$q
  timeout -k 10 300 python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --extra C2F,C4 > "$O/bench_${TAG}_q$q.json" 2> "$O/bench_${TAG}_q$q.err" \
    || { echo "bench q$q failed"; tail -5 "$O/bench_${TAG}_q$q.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('q$q', d['value'], d['ms_per_step'], d['config'].get('frame_ms_one_stream'), [(e.get('config'), e.get('frame_ms')) for e in d.get('extra', [])])" "$O/bench_${TAG}_q$q.json"
done
