# bench.py at the driver's short settings (--steps 20 --warmup 5) with and without the pre-warmup re-settle,
# interleaved, C2 only; then two steady-state lines. Results: gpurun_out/short20*.jsonl, long200.jsonl
set -u
mkdir -p gpurun_out
for i in 1 2 3; do
  for rs in 0 30; do
    timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --extra= --no-cpu-baseline --resettle-ms $rs \
      >> gpurun_out/short20_rs$rs.jsonl 2>/dev/null || exit 1
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/short20_rs*.jsonl")):
    for l in open(f):
        d=json.loads(l); print(f, d["value"], d["ms_per_step"], d["config"]["frames_in_flight"], d["config"]["in_flight_ms_rank0"])
PY
