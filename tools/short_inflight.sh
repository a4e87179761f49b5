# bench.py at the driver's short settings (--steps 20 --warmup 5, C2 only) with 2, 3, 4 frames in flight forced,
# interleaved, 3 rounds: which count a 20-frame region prefers. Results: gpurun_out/short_if*.jsonl
set -u
mkdir -p gpurun_out
for i in 1 2 3; do
  for s in 2 3 4; do
    timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --extra= --no-cpu-baseline --in-flight $s \
      >> gpurun_out/short_if$s.jsonl 2>/dev/null || exit 1
  done
done
python3 - <<'PY'
import json, glob, statistics
for f in sorted(glob.glob("gpurun_out/short_if*.jsonl")):
    v = [json.loads(l)["value"] for l in open(f)]
    print(f, [round(x) for x in v], "median", round(statistics.median(v)))
PY
