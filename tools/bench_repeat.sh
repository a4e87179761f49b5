#!/bin/bash
# Repeatability and resolution sweep of the headline bench (run on the GPU box from the repo root):
#   bash tools/bench_repeat.sh  -> gpurun_out/bench_repeat/{run*,size*}.json
set -e
O=gpurun_out/bench_repeat; mkdir -p $O
for k in 1 2 3; do
  timeout -k 10 300 python3 bench.py --steps 400 --warmup 100 --extra= --no-cpu-baseline > $O/run$k.json 2> $O/run$k.err
  python3 -c "import json; d=json.load(open('$O/run$k.json')); print('run $k', d['value'], d['ms_per_step'], d['config']['frame_ms_one_stream'])"
done
for s in 1280x720 2560x1440 3840x2160; do
  timeout -k 10 300 python3 bench.py --steps 200 --warmup 50 --size $s --extra= --no-cpu-baseline > $O/size_$s.json 2> $O/size_$s.err
  python3 -c "import json; d=json.load(open('$O/size_$s.json')); print('size $s', d['value'], d['ms_per_step'], d['config']['frame_ms_one_stream'])"
done
