"""Summarises RT_PHASE_TIMING=1 output (PH <primary trace> <hit shading> <shadow traces + store>)."""
import sys
import statistics
rows = [list(map(int, ln.split()[1:4])) for ln in open(sys.argv[1]) if ln.startswith("PH ")]
if not rows:
    sys.exit("no PH lines")
tot = [sum(r) for r in rows]
for k, name in enumerate(["primary trace", "hit shading", "shadow traces"]):
    v = [r[k] for r in rows]
    print(f"{name:14s} mean {statistics.mean(v):9.0f} median {statistics.median(v):9.0f} "
          f"share {sum(v) / sum(tot):.3f}")
print(f"waves sampled {len(rows)}; per wave total mean {statistics.mean(tot):.0f} cycles")
