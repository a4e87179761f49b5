#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy table of a HIP source (hipcc -Rpass-analysis=
kernel-resource-usage), e.g.  python3 tools/kres.py realtimeraytracing_gradproject_amd/csrc/rt_trace.hip [-DX=1]"""
import re
import subprocess
import sys

src, extra = sys.argv[1], sys.argv[2:]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
       "-munsafe-fp-atomics", "-c", src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"] + extra
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for ln in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", ln)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        name = t.split(":", 1)[1].strip()
        dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        dm = re.sub(r"rt::\(anonymous namespace\)::", "", dm)
        dm = dm.split("(")[0]
        cur = {"name": dm}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
keys = ["VGPRs", "AGPRs", "SGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "SGPRs Spill", "VGPRs Spill",
        "LDS Size [bytes/block]"]
print(f"{'kernel':60s} " + " ".join(f"{k.split()[0][:8]:>8s}" for k in keys))
for r in rows:
    if len(sys.argv) > 1 and "--all" not in extra and "k_" not in r["name"]:
        continue
    print(f"{r['name'][:60]:60s} " + " ".join(f"{r.get(k, '-'):>8s}" for k in keys))
