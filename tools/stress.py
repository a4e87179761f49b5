#!/usr/bin/env python3
"""Stress run of the library (production hardening, not a benchmark): for a wall-clock budget it keeps the GPU busy
with randomised work and checks results as it goes.

Each episode picks a scene (the BASELINE configs, REF / REFL, DEGEN and seeded random scenes of
tests/random_scenes.py) at a random size, a tile-balance mode (plain, adaptive, forced 2..5), a tile height (8 or 4),
1..4 render streams and a run of frames with a camera moving every frame; grid scenes move their instances with
per-frame TLAS updates (update_only) while frames are in flight; some episodes go through the tiled multi-GPU loop on
the loopback transport (N = 2..8, 1..4 frames per launch). Checks:
  * every K-th frame is rendered again with the other schedule (per lane vs packet) and must be bit-identical;
  * a few frames per episode, at reduced size, must equal the CPU oracle bit for bit;
  * the tile plan's cover check (RT_BALANCE_CHECK) must never fail and no plan may refuse items under adaptive mode.
Prints a progress line every ~20 s and a JSON summary at the end; exits non-zero on the first mismatch.

  python3 tools/stress.py --minutes 8 [--seed 1]
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

os.environ["RT_BALANCE_CHECK"] = "1"  # read at context creation
import realtimeraytracing_gradproject_amd as rt  # noqa: E402
from realtimeraytracing_gradproject_amd import scenes  # noqa: E402

import oracle  # noqa: E402
from random_scenes import random_scene  # noqa: E402

NAMES = ["C2", "C2F", "C3", "C4", "C5", "REF", "REFL", "DEGEN", "RANDOM"]


def pick_scene(rng):
    name = NAMES[int(rng.integers(0, len(NAMES)))]
    if name == "RANDOM":
        spec = random_scene(int(rng.integers(0, 1 << 30)), width=160, height=90)
    else:
        spec = scenes.config(name)
    scale = float(rng.choice([0.125, 0.25, 0.5])) if name != "C5" else float(rng.choice([0.05, 0.1]))
    w = max(1, int(spec.width * scale) + int(rng.integers(-3, 4)))
    h = max(1, int(spec.height * scale) + int(rng.integers(-3, 4)))
    return name, spec.with_size(w, h)


def moved(spec, k, n, wobble):
    (ex, ey, ez), tgt, up = spec.camera
    r = math.hypot(ex - tgt[0], ez - tgt[2]) or 1.0
    a = math.atan2(ez - tgt[2], ex - tgt[0]) + wobble * 2.0 * math.pi * k / max(n, 1)
    sp = spec.with_size(spec.width, spec.height)
    sp.camera = ((tgt[0] + r * math.cos(a), ey * (0.7 + 0.3 * math.cos(3.0 * a)), tgt[2] + r * math.sin(a)), tgt, up)
    return sp


def instances_at(spec, ids, k):
    """Grid scenes: every model instance bobs in y with frame k (translation only), the plane stays."""
    out = []
    for (m, x, iid, hg) in spec.instances:
        x = np.array(x, np.float32).copy()
        if hg == rt.RT_HITGROUP_MODEL and len(spec.instances) > 8:
            x[7] += 0.25 * math.sin(0.3 * k + 0.7 * iid)
        out.append((ids[m], x, iid, hg))
    return out


def render(c, spec, stream, schedule=None):
    if schedule is not None:
        c.set_schedule(schedule)
    out = torch.empty((spec.height, spec.width, 4), dtype=torch.uint8, device="cuda")
    c.dispatch(spec.width, spec.height, out, stream=stream.cuda_stream)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--minutes", type=float, default=8.0)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    rng = np.random.default_rng(a.seed)
    t_end = time.time() + a.minutes * 60.0
    t_print = time.time()
    tally = {"episodes": 0, "frames": 0, "schedule_checks": 0, "oracle_checks": 0, "loopback_episodes": 0,
             "tlas_updates": 0, "hot_reloads": 0, "limit_refusals": 0, "batch_episodes": 0, "plans": 0,
             "by_scene": {}}
    while time.time() < t_end:
        name, spec = pick_scene(rng)
        tally["episodes"] += 1
        tally["by_scene"][name] = tally["by_scene"].get(name, 0) + 1
        c = rt.Context(0)
        ids = scenes.upload(c, spec)
        mode = int(rng.choice([0, 1, 1, 1, 2, 3, 4, 5]))
        c.set_tile_balance(mode)
        rows4 = bool(rng.random() < 0.25)
        if rows4:
            c.set_tile_rows(4)
        n = int(rng.integers(8, 80))
        wobble = float(rng.uniform(0.05, 1.0))
        grid = len(spec.instances) > 8 and name != "RANDOM"
        if rng.random() < 0.12:
            # batches (rt_dispatch_frames: 1..4 frames, a camera each) on 1..3 streams, rt_trace_rays launched on
            # another stream between them; sampled frames == a single rt_dispatch_rays of the same camera, the rays'
            # hits == the same rays traced again alone
            tally["batch_episodes"] += 1
            nstreams = int(rng.integers(1, 4))
            streams = [torch.cuda.Stream() for _ in range(nstreams)]
            sr = torch.cuda.Stream()
            nray = 4096
            o_ = rng.normal(size=(nray, 3))
            o_ = o_ / np.linalg.norm(o_, axis=1, keepdims=True) * 20.0
            d_ = rng.uniform(-3, 3, size=(nray, 3)) - o_
            d_ /= np.linalg.norm(d_, axis=1, keepdims=True)
            rays = np.zeros((nray, 8), np.float32)
            rays[:, :3], rays[:, 4:7], rays[:, 7] = o_, d_, 1e5
            d_rays = torch.from_numpy(rays).cuda()
            hits_a = torch.zeros((nray, 4), dtype=torch.int32, device="cuda")
            batches, specs = [], []
            for k0 in range(0, n, 4):
                F = int(rng.integers(1, 5))
                sps = [moved(spec, k, n, wobble) for k in range(k0, k0 + F)]
                buf = torch.empty((F, spec.height, spec.width, 4), dtype=torch.uint8, device="cuda")
                cams = np.stack([sp.camera_buffer().ravel() for sp in sps])
                try:
                    c.dispatch_frames(spec.width, spec.height, buf, cams, stream=streams[(k0 // 4) % nstreams].cuda_stream)
                except rt.RtError as e:
                    if "forced layouts take at most" not in str(e):
                        raise
                    tally["limit_refusals"] += 1  # the documented cap of the test-only forced layouts
                    c.set_tile_balance(1)
                    c.dispatch_frames(spec.width, spec.height, buf, cams, stream=streams[(k0 // 4) % nstreams].cuda_stream)
                batches.append(buf)
                specs.append(sps)
                if k0 == 0:
                    any_hit = bool(rng.random() < 0.5)
                    c.trace_rays(d_rays, nray, any_hit, hits_a, stream=sr.cuda_stream)
            torch.cuda.synchronize()
            tally["frames"] += sum(len(x) for x in specs)
            hits_b = torch.zeros((nray, 4), dtype=torch.int32, device="cuda")
            c.trace_rays(d_rays, nray, any_hit, hits_b, stream=sr.cuda_stream)
            torch.cuda.synchronize()
            if not torch.equal(hits_a, hits_b):
                print(json.dumps({"error": "rays traced beside frames != traced alone", "scene": name}), flush=True)
                return 1
            for q in sorted(set(int(x) for x in rng.integers(0, len(batches), size=2))):
                j = int(rng.integers(0, len(specs[q])))
                c.set_camera(specs[q][j].camera_buffer())
                ref = render(c, specs[q][j], streams[0], rt.RT_SCHED_PACKET)
                torch.cuda.synchronize()
                if not torch.equal(ref, batches[q][j]):
                    print(json.dumps({"error": "batched frame != dispatch", "scene": name, "batch": q, "frame": j,
                                      "mode": mode}), flush=True)
                    return 1
                tally["schedule_checks"] += 1
        elif rng.random() < 0.2 and spec.width >= 8 and spec.height >= 8:
            # the tiled loop on the loopback transport, a camera per frame
            tally["loopback_episodes"] += 1
            nranks = int(rng.integers(2, 9))
            comm = rt.Comm.loopback(c, nranks)
            fpl = int(rng.integers(1, 5))
            comm.set_batch(fpl)
            frames, specs = [], []
            for k0 in range(0, n, fpl):
                m = min(fpl, n - k0)
                sps = [moved(spec, k, n, wobble) for k in range(k0, k0 + m)]
                fs = [torch.empty((spec.height, spec.width, 4), dtype=torch.uint8, device="cuda") for _ in range(m)]
                try:
                    comm.render_strips_frames(spec.width, spec.height, fs,
                                              np.concatenate([sp.camera_buffer().ravel() for sp in sps]))
                except rt.RtError as e:
                    # the test-only forced layouts cap a launch at 32768 waves (rt_set_tile_balance): a documented
                    # refusal, reported by the call, not a fault; the episode goes on without the forced layout
                    if "forced layouts take at most" not in str(e):
                        raise
                    tally["limit_refusals"] += 1
                    c.set_tile_balance(1)
                    comm.render_strips_frames(spec.width, spec.height, fs,
                                              np.concatenate([sp.camera_buffer().ravel() for sp in sps]))
                frames += fs
                specs += sps
            comm.synchronize()
            comm.close()
            tally["frames"] += n
            # the loop's frames against the plain dispatch of the same camera (same context, packet schedule)
            s0 = torch.cuda.Stream()
            for k in sorted(set(int(x) for x in rng.integers(0, n, size=3))):
                c.set_camera(specs[k].camera_buffer())
                ref = render(c, specs[k], s0, rt.RT_SCHED_PACKET)
                torch.cuda.synchronize()
                if not torch.equal(ref, frames[k]):
                    print(json.dumps({"error": "loopback frame != dispatch", "scene": name, "frame": k,
                                      "nranks": nranks, "fpl": fpl, "mode": mode}), flush=True)
                    return 1
                tally["schedule_checks"] += 1
        else:
            nstreams = int(rng.integers(1, 5))
            streams = [torch.cuda.Stream() for _ in range(nstreams)]
            outs, specs = [], []
            # hot reload: mesh 0 rebuilt with displaced vertices halfway through, a full TLAS build
            # after it, frames of the old and the new mesh in flight around it on the episode's streams
            reload_at = n // 2 if (not grid and rng.random() < 0.15) else None
            for k in range(n):
                sp = moved(spec, k, n, wobble)
                c.set_camera(sp.camera_buffer())
                if grid and k % 5 == 4:
                    c.tlas_build(instances_at(spec, ids, k), update_only=True)
                    tally["tlas_updates"] += 1
                if reload_at is not None and k == reload_at:
                    v0, i0 = spec.meshes[0]
                    v1 = np.array(v0, np.float32).copy()
                    v1[:, :3] += rng.normal(scale=0.02, size=(v1.shape[0], 3)).astype(np.float32)
                    c.blas_rebuild(ids[0], v1, i0)
                    c.tlas_build([(ids[m], x, iid, hg) for (m, x, iid, hg) in spec.instances])
                    spec = scenes.SceneSpec(**{**spec.__dict__})
                    spec.meshes = [(v1, i0)] + list(spec.meshes[1:])
                    tally["hot_reloads"] += 1
                outs.append((render(c, sp, streams[k % nstreams]), k))
                specs.append(sp)
            torch.cuda.synchronize()
            tally["frames"] += n
            # other-schedule re-renders of a few frames, the scene state at that frame restored first
            s0 = streams[0]
            lo = reload_at if reload_at is not None else 0  # frames before a reload saw the old mesh
            for k in sorted(set(int(x) for x in rng.integers(lo, n, size=2))):
                last = ((k - 4) // 5) * 5 + 4 if k >= 4 else None
                if grid:  # the instances as frame k saw them: the last update at an index = 4 (mod 5) up to k
                    c.tlas_build(instances_at(spec, ids, last) if last is not None else
                                 [(ids[m], x, iid, hg) for (m, x, iid, hg) in spec.instances], update_only=True)
                c.set_camera(specs[k].camera_buffer())
                lane = render(c, specs[k], s0, rt.RT_SCHED_LANE)
                torch.cuda.synchronize()
                c.set_schedule(rt.RT_SCHED_PACKET)
                if not torch.equal(lane, outs[k][0]):
                    # the schedules must agree (packet_tri's own-box mask); on a mismatch report which
                    # side departs from the oracle's emulation of its schedule, and the packet frame rendered again
                    # now (nothing else in flight)
                    again = render(c, specs[k], s0, rt.RT_SCHED_PACKET)
                    torch.cuda.synchronize()
                    sk = scenes.SceneSpec(**{**spec.__dict__})
                    if grid:  # the instances frame k saw (the oracle builds that TLAS afresh; the GPU refitted it)
                        sk.instances = [(m, x, iid, hg) for (m, (_, x, iid, hg)) in
                                        zip([i[0] for i in spec.instances],
                                            instances_at(spec, ids, last) if last is not None else
                                            [(ids[m], x, iid, hg) for (m, x, iid, hg) in spec.instances])]
                    o = oracle.Scene(sk)
                    per_ray = o.render_spec(specs[k], nthreads=8, want_float=False, schedule=1)[0]
                    packet = o.render_spec(specs[k], nthreads=8, want_float=False, schedule=0)[0]
                    g_lane, g_pk, g_again = lane.cpu().numpy(), outs[k][0].cpu().numpy(), again.cpu().numpy()
                    diff = np.argwhere((g_lane != g_pk).any(axis=2))
                    print(json.dumps({"error": "lane schedule != packet frame", "scene": name, "frame": k,
                                      "mode": mode, "streams": nstreams, "size": [specs[k].width, specs[k].height],
                                      "camera": specs[k].camera, "tile_rows4": rows4, "pixels": len(diff),
                                      "grid_update": last if grid else None, "seed_episode": tally["episodes"],
                                      "first": diff[:6].tolist(),
                                      "lane==oracle_per_ray": bool(np.array_equal(g_lane, per_ray)),
                                      "packet==oracle_packet": bool(np.array_equal(g_pk, packet)),
                                      "packet_again==oracle_packet": bool(np.array_equal(g_again, packet)),
                                      "oracle_packet==oracle_per_ray": bool(np.array_equal(packet, per_ray))}),
                          flush=True)
                    return 1
                tally["schedule_checks"] += 1
        info = c.tile_balance_info()
        tally["plans"] += int(info["plans"])
        if info["check_bad"] != 0 or (mode == 1 and info["refused"] != 0):
            print(json.dumps({"error": "tile plan check", "scene": name, "info": info}), flush=True)
            return 1
        # one oracle check per episode at reduced size (the CPU oracle is the slow side)
        if not grid or rng.random() < 0.5:
            sp = spec.with_size(min(spec.width, 96), min(spec.height, 64))
            if grid:
                c.tlas_build([(ids[m], x, iid, hg) for (m, x, iid, hg) in spec.instances], update_only=True)
            c.set_camera(sp.camera_buffer())
            c.set_tile_balance(int(rng.choice([0, 1, 2, 5])))
            got = render(c, sp, torch.cuda.Stream(), rt.RT_SCHED_PACKET)
            torch.cuda.synchronize()
            want, _, _ = oracle.Scene(spec).render_spec(sp, nthreads=8, want_float=False)
            if not np.array_equal(got.cpu().numpy(), want):
                print(json.dumps({"error": "frame != oracle", "scene": name, "size": [sp.width, sp.height],
                                  "camera": sp.camera}), flush=True)
                return 1
            tally["oracle_checks"] += 1
        c.close()
        if time.time() - t_print > 20:
            t_print = time.time()
            print(json.dumps({"progress": {k: v for k, v in tally.items() if k != "by_scene"}}), flush=True)
    print(json.dumps({"stress": "ok", "minutes": a.minutes, "seed": a.seed, **tally}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
