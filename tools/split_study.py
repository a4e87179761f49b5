#!/usr/bin/env python3
"""Design study (CPU): would tracing the costliest 8 x 8 tiles as several smaller sub-packets, dispatched first,
shorten the launch? tools/split_study.c gives each tile's packet fetches (the kernel's cost unit: the measured wave
time correlates 0.92 with them on C4, tools/tile_study.py) for the full packet and for its 8x4 / 4x4 / 2x2
sub-packets. A list-scheduling model of the launch (7 wave slots per SIMD, 1024 SIMDs, waves dispatched in grid
order to the earliest free slot, duration = fetches x the C4-calibrated us per fetch) then compares:
  base        - every tile one wave, row-major grid order (the shipped kernel)
  split<k>@q  - tiles above the q-quantile of cost traced as k sub-packets (k = 2, 4, 16), those sub-waves first
                in the grid (costliest first), then every other tile in row-major order
for the whole frame and for rank 0's share at N ranks (interleaved 8-row strips).
  python3 tools/split_study.py --config C4 --shares 1,4,8"""
import argparse
import ctypes
import heapq
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SLOTS = 256 * 4 * 7


def costs(config: str, nthreads: int):
    cache = f"/tmp/split_{config}.npy"
    if os.path.exists(cache):
        return np.load(cache)
    so = "/tmp/libsplit.so"
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-ffp-contract=off", "-mfma", "-o", so,
                    os.path.join(ROOT, "tools", "split_study.c"), "-lm", "-lpthread"], check=True)
    import oracle
    lib = ctypes.CDLL(so)
    for n, r, args in oracle._SIGS:
        if hasattr(lib, n):
            f = getattr(lib, n)
            f.restype, f.argtypes = r, args
    oracle.lib = lib
    from realtimeraytracing_gradproject_amd import scenes
    spec = scenes.config(config)
    W, H = spec.width, spec.height
    sc = oracle.Scene(spec)
    cb = (ctypes.c_float * 64)(*[float(x) for x in spec.camera_buffer().ravel()])
    lights = oracle._lights(spec.lights)
    tw, th = W // 8, H // 8
    out = np.zeros((th, tw, 23), np.uint64)
    lib.split_study(ctypes.c_void_p(sc._h), cb, lights, len(spec.lights), W, H, nthreads,
                    out.ctypes.data_as(ctypes.c_void_p))
    np.save(cache, out)
    return out


def makespan(durs):
    """List scheduling in order onto SLOTS wave slots."""
    heap = [0.0] * SLOTS
    end = 0.0
    for d in durs:
        t = heapq.heappop(heap)
        e = t + d
        end = max(end, e)
        heapq.heappush(heap, e)
    return end


def plan(c, k, q):
    """Durations in dispatch order: tiles above the cost quantile q as k sub-packets, costliest first."""
    full = c[..., 0].ravel().astype(float)
    col = {1: [0], 2: [1, 2], 4: [3, 4, 5, 6], 16: list(range(7, 23))}[k]
    sub = c.reshape(-1, 23)[:, col].astype(float)
    thr = np.quantile(full, q) if q < 1 else np.inf
    heavy = full > thr
    front = np.sort(sub[heavy].ravel())[::-1]
    rest = full[~heavy]
    return np.concatenate([front, rest]), int(heavy.sum()), float(sub[heavy].sum() / max(full[heavy].sum(), 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--shares", default="1,4,8")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--us-per-fetch", type=float, default=0.0,
                    help="0: calibrate an affine wave time a + b x fetches to the measured C4 wave mean (42.5 us) and "
                         "longest wave (246 us, profiles/r03_wave_times_C4.txt)")
    ap.add_argument("--us-per-wave", type=float, default=-1.0, help="the affine model's fixed part a (-1: calibrate)")
    a = ap.parse_args()
    c = costs(a.config, a.threads)
    th, tw = c.shape[:2]
    full = c[..., 0].astype(float)
    upf = a.us_per_fetch or (246.4 - 42.48) / (full.max() - full.mean())
    fixed = a.us_per_wave if a.us_per_wave >= 0 else 42.48 - upf * full.mean()
    print(f"{a.config}: {th * tw} tiles, fetches per tile mean {full.mean():.1f} p90 {np.quantile(full, 0.9):.0f} "
          f"max {full.max():.0f}; wave time {fixed:.2f} us + {upf:.4f} us per fetch")

    def us(f):
        return fixed + upf * f
    for q in (2, 4, 16):
        ratio = c.reshape(-1, 23)[:, {2: [1, 2], 4: [3, 4, 5, 6], 16: list(range(7, 23))}[q]].max(axis=1) / np.maximum(
            c[..., 0].ravel(), 1)
        top = np.argsort(-full.ravel())[:200]
        print(f"  {q} sub-packets: costliest sub-packet / full packet over the 200 costliest tiles: "
              f"median {np.median(ratio[top]):.3f}, max {ratio[top].max():.3f}")
    for share in [int(x) for x in a.shares.split(",")]:
        rows = [r for r in range(th) if r % share == 0]  # rank 0's 8-row strips = tile rows r % N == 0
        cs = c[rows]
        base = makespan(us(cs[..., 0].ravel().astype(float)))
        print(f"share N={share}: {len(rows) * tw} waves; base makespan {base:.1f} us, longest wave "
              f"{us(cs[..., 0].max()):.1f} us")
        for k in (2, 4, 16):
            for q in (0.99, 0.97, 0.95, 0.9, 0.8):
                durs, nh, work = plan(cs, k, q)
                ms = makespan(us(durs))
                print(f"  split{k}@{q}: {nh} tiles split (sub-packets cost {work:.2f}x their tiles), waves "
                      f"{len(durs)}, makespan {ms:.1f} us ({ms / base:.3f}), longest {us(durs.max()):.1f} us")
        durs = np.sort(cs[..., 0].ravel().astype(float))[::-1]
        print(f"  longest-first order only: {makespan(us(durs)):.1f} us")
        # adaptive: the launch's load bound L = summed wave time / wave slots; a tile whose wave would outlast
        # alpha x L is split into the fewest sub-packets (4, else 16) whose costliest part fits, and every wave is
        # dispatched longest first (a counting sort by cost)
        flat = cs.reshape(-1, 23).astype(float)
        for alpha in (0.5, 0.75, 1.0, 1.5):
            L = us(flat[:, 0]).sum() / SLOTS
            items = []
            nsplit = 0
            for row in flat:
                if us(row[0]) <= alpha * L:
                    items.append(row[0])
                    continue
                nsplit += 1
                q4, q16 = row[3:7], row[7:23]
                items.extend(q4 if us(q4.max()) <= alpha * L or us(q16.max()) >= us(q4.max()) else q16)
            d = np.sort(np.array(items))[::-1]
            ms = makespan(us(d))
            print(f"  adaptive alpha {alpha}: L {L:.1f} us, {nsplit} tiles split, waves {len(d)}, longest-first "
                  f"makespan {ms:.1f} us ({ms / base:.3f}), longest {us(d.max()):.1f} us")
        # the kernel's rule (the plan kernel only knows whole-tile costs): T = beta x L; a tile costing more than T
        # becomes 4 sub-packets when 0.55 x its cost (the median costliest quadrant) fits T, else 16; waves ordered
        # by estimated cost (tile cost x 0.55 / 0.35 for parts), longest first
        for beta in (0.3, 0.35, 0.4, 0.5):
            wt = us(flat[:, 0])
            L = wt.sum() / SLOTS
            T = max(L, beta * wt.max())
            est, act = [], []
            nsplit = 0
            for row, cw in zip(flat, wt):
                if cw <= T:
                    est.append(cw)
                    act.append(row[0])
                    continue
                nsplit += 1
                if 0.55 * cw <= T:
                    est.extend([0.55 * cw] * 4)
                    act.extend(row[3:7])
                else:
                    est.extend([0.35 * cw] * 16)
                    act.extend(row[7:23])
            order = np.argsort(-np.array(est), kind="stable")
            d = np.array(act)[order]
            ms = makespan(us(d))
            print(f"  rule T = max(L, {beta} x costliest): T {T:.1f} us, {nsplit} tiles split, waves {len(d)}, makespan {ms:.1f} us "
                  f"({ms / base:.3f}), longest {us(d.max()):.1f} us")


if __name__ == "__main__":
    main()
