set -u
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --extra= --no-cpu-baseline >> gpurun_out/short20.jsonl 2>/dev/null || exit 1
done
for i in 1 2; do
  timeout -k 10 120 python3 bench.py --steps 200 --warmup 100 --extra= --no-cpu-baseline >> gpurun_out/long200.jsonl 2>/dev/null || exit 1
done
python3 - <<'PY'
import json
for f in ("gpurun_out/short20.jsonl","gpurun_out/long200.jsonl"):
    for l in open(f):
        d=json.loads(l); print(f, d["value"], d["ms_per_step"], d["config"]["frames_in_flight"], d["config"]["in_flight_ms_rank0"], d["config"]["frame_ms_one_stream"])
PY
