"""Per-wave start / end clocks of one frame (library built with -DRT_WAVE_TIMES=1): occupancy over
time, the launch's ramp and tail, per-XCD finish times.
  python tools/wave_times.py --lib <variant .so> --config C2"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import realtimeraytracing_gradproject_amd as rt  # noqa: E402
from realtimeraytracing_gradproject_amd import scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", required=True)
ap.add_argument("--config", default="C2")
ap.add_argument("--frames", type=int, default=30)
ap.add_argument("--balance", type=int, default=1, help="rt_set_tile_balance mode (0: the plain grid)")
ap.add_argument("--share", type=int, default=1, help="rank 0's interleaved 8-row strips of a frame over N ranks")
a = ap.parse_args()
spec = scenes.config(a.config)
c = rt.Context(0, library=rt._load(a.lib))
scenes.upload(c, spec)
c.set_tile_balance(a.balance)
W, H = spec.width, spec.height
rows = None if a.share == 1 else rt.strip_rows(H, a.share, 0)
NR = H if rows is None else len(rows)
out = torch.zeros((NR, W, 4), dtype=torch.uint8, device="cuda")
tb = torch.zeros((NR * W * 4,), dtype=torch.float32, device="cuda")  # 16 B per pixel: room for every wave record
s = torch.cuda.current_stream().cuda_stream
for _ in range(a.frames):
    c.dispatch(W, H, out, tb.view(NR, W, 4), rows=rows, stream=s)
torch.cuda.synchronize()
tb.zero_()
c.dispatch(W, H, out, tb.view(NR, W, 4), rows=rows, stream=s)
torch.cuda.synchronize()
u = tb.view(torch.int32).cpu().numpy().astype(np.uint32).reshape(-1, 4)
live = u[:, 1] != 0
u = u[live]
t0 = u[:, 0].astype(np.int64)
t1 = u[:, 1].astype(np.int64)
base = t0.min()
t0 -= base
t1 -= base
T = t1.max()
print(f"{a.config} share 1/{a.share}: {len(u)} waves, frame {T * 10 / 1000:.1f} us (100 MHz clock), tile balance {a.balance}: "
      f"{c.tile_balance_info()}")
dur = (t1 - t0) * 10 / 1000
print(f"wave duration us: mean {dur.mean():.2f} p50 {np.median(dur):.2f} p90 {np.percentile(dur, 90):.2f} "
      f"max {dur.max():.2f}")
# occupancy over time in 20 bins
edges = np.linspace(0, T, 21)
occ = []
for k in range(20):
    lo, hi = edges[k], edges[k + 1]
    ov = np.clip(np.minimum(t1, hi) - np.maximum(t0, lo), 0, None).sum() / (hi - lo)
    occ.append(ov)
print("resident waves per 5% of the frame:", " ".join(f"{o:.0f}" for o in occ))
print(f"mean resident {np.mean(occ):.0f}; last wave start at {t0.max() * 10 / 1000:.1f} us")
xcc = u[:, 2] & 0xf
for x in range(8):
    m = xcc == x
    if m.any():
        print(f"XCC {x}: waves {m.sum()} last end {t1[m].max() * 10 / 1000:.1f} us mean dur {dur[m].mean():.2f} us")
# residency: the instantaneous peak of resident waves (a sweep over the start / end events, not a bin
# mean), and where the waves sat: HW_ID (gfx9 layout) = wave slot [3:0], SIMD [5:4], CU [11:8], SH [12], SE [15:13]
hw = u[:, 3]
simd_key = (xcc.astype(np.int64) << 16) | ((hw >> 8) & 0xff).astype(np.int64) << 4 | ((hw >> 4) & 3)
cu_key = simd_key >> 2
ev_t = np.concatenate([t0, t1])
ev_d = np.concatenate([np.ones_like(t0), -np.ones_like(t1)])
order = np.lexsort((ev_d, ev_t))  # ends before starts at equal clocks
peak = int(np.cumsum(ev_d[order]).max())
per_simd = []
for key in np.unique(simd_key):
    m = simd_key == key
    et = np.concatenate([t0[m], t1[m]])
    ed = np.concatenate([np.ones(m.sum(), np.int64), -np.ones(m.sum(), np.int64)])
    o = np.lexsort((ed, et))
    per_simd.append(int(np.cumsum(ed[o]).max()))
per_simd = np.array(per_simd)
slot_ids = np.unique(hw & 0xf)
print(f"residency: peak {peak} waves at once; {len(np.unique(cu_key))} CUs, {len(per_simd)} SIMDs seen; most waves at "
      f"once on one SIMD {per_simd.max()} (SIMDs reaching it: {(per_simd == per_simd.max()).sum()}); HW wave slot ids "
      f"used {slot_ids.min()}..{slot_ids.max()}; the plan's load-bound slots (rt_tile_balance_info[15]): "
      f"{c.tile_balance_info().get('slots')}")
np.savez(os.path.join(ROOT, "gpurun_out", f"wt_{a.config}_n{a.share}_b{a.balance}.npz"), t0=t0, t1=t1, ids=np.nonzero(live)[0], xcc=xcc,
         hw=hw)
c.close()
