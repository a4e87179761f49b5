#!/usr/bin/env python3
"""Headline benchmark: Mrays/s (primary + shadow) at 1080p on MI355X — BASELINE.json config C2
(teapot.obj, 1 light, 1920x1080, primary + shadow rays) by default.

A step is one frame: RayGen -> TLAS/BLAS traversal -> shading + shadow rays -> RGBA8 (the
reference's DispatchRays, D3D12HelloTriangle.cpp:558-592). The scene is static: the LBVH build
runs once before the timed region and is reported separately (build_ms).

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): every pixel is an
independent unit, so the job shards with no data-path collective. Default ("frames"): a step is a
batch of N frames of the configured view, one per rank, each left in its rank's HBM (per-GPU work
fixed: scaling "weak"). --assemble instead splits ONE frame into interleaved 8-row strips (strip s
-> rank s mod N), gathers them to rank 0 over RCCL and un-interleaves them there
(rt_assemble_strips): scaling "strong", the presentation path of a single-view frame.

value = rays traced in one step (all ranks, counted by the device counters in an untimed pass)
x steps / max-over-ranks wall time of the timed region.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import realtimeraytracing_gradproject_amd as rt  # noqa: E402
from realtimeraytracing_gradproject_amd import distributed as D, scenes  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
L2_PEAK_GBS = 34500.0  # aggregate L2 bandwidth, 8 XCDs (MI355X_MICROARCH.md, L2 section)
BYTES_PER_AABB_TEST = 24  # one child box (6 floats) per slab test
BYTES_PER_TRI_TEST = 36   # v0, e1, e2 (9 floats) per Moller-Trumbore test
BYTES_PER_PIXEL = 4       # RGBA8 write
STRIP_ROWS = D.STRIP_ROWS


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=100,
                   help="untimed frames first: the GPU needs ~20 ms of load to reach steady clocks")
    p.add_argument("--config", default="C2", choices=[c for c in scenes.CONFIGS])
    p.add_argument("--schedule", default="packet", choices=["packet", "lane"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="minimum wall time of the CPU baseline sample")
    p.add_argument("--assemble", action="store_true",
                   help="N>1: split one frame into strips and gather it to rank 0 (strong scaling)")
    p.add_argument("--save-image", default="", help="write the rank-0 frame as .npy")
    p.add_argument("--extra", default="C2F,C3,C4,C5,REF",
                   help="comma list of further configs timed on one GPU (N=1 only; '' to skip)")
    return p.parse_args()


def load_traffic(config: str):
    """HBM bytes per trace launch from the committed rocprofv3 PMC pass (profiles/), if present."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(config)
        return float(e["bytes_per_launch"]) if e else None
    except Exception:
        return None


def cpu_baseline(spec, seconds: float):
    """The oracle (scalar C, pthreads over interleaved rows) on the same frame, on this host."""
    import oracle

    ncpu = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    threads = max(1, min(16, ncpu or 1))
    o = oracle.Scene(spec)
    rays = 0
    frames = 0
    t0 = time.perf_counter()
    while True:
        _, _, st = o.render_spec(spec, nthreads=threads, want_float=False, schedule=1)  # per-ray: the CPU form
        rays += int(st[0] + st[1])
        frames += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            break
    # also one thread, and the host CPU model
    t1 = time.perf_counter()
    _, _, st1 = o.render_spec(spec, nthreads=1, want_float=False, schedule=1)
    dt1 = time.perf_counter() - t1
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), None)
    except OSError:
        pass
    return {"value": rays / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{frames} full {spec.name} frame(s) {spec.width}x{spec.height} by oracle/rt_oracle.c "
                      f"({threads} threads, {dt:.1f} s wall)",
            "single_thread": round(int(st1[0] + st1[1]) / dt1 / 1e6, 3), "host_cpus": ncpu, "cpu_model": model}


def measure_config(name: str, steps: int, warmup: int, schedule: int) -> dict:
    """Single-GPU frame rate of another BASELINE config (reported under "extra", not the headline)."""
    spec = scenes.config(name)
    W, H = spec.width, spec.height
    with rt.Context(torch.cuda.current_device()) as ctx:
        scenes.upload(ctx, spec)
        ctx.set_schedule(schedule)
        stream = torch.cuda.Stream()
        out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
        ctx.set_stats(True)
        ctx.stats_reset()
        ctx.dispatch(W, H, out, None, stream=stream.cuda_stream)
        torch.cuda.synchronize()
        st = ctx.stats()
        ctx.set_stats(False)
        for _ in range(warmup):
            ctx.dispatch(W, H, out, None, stream=stream.cuda_stream)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(steps):
            ctx.dispatch(W, H, out, None, stream=stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        ms = e0.elapsed_time(e1) / steps
    rays = st["primary_rays"] + st["shadow_rays"]
    return {"config": name, "Mrays_s": round(rays * steps / wall / 1e6, 1), "frame_ms": round(wall / steps * 1e3, 4),
            "kernel_ms": round(ms, 4), "rays_per_frame": int(rays), "resolution": f"{W}x{H}", "spp": spec.spp,
            "aabb_tests_per_ray": round(st["aabb_tests"] / max(rays, 1), 2),
            "tri_tests_per_ray": round(st["tri_tests"] / max(rays, 1), 2)}


def measure_raster(name: str, steps: int, warmup: int) -> dict:
    """Raster fallback (rt_raster_draw: the reference's scrapped raster pipeline, model + plane with
    instance 0's transform) on one GPU, reported under "extra"."""
    spec = scenes.config(name)
    W, H = spec.width, spec.height
    with rt.Context(torch.cuda.current_device()) as ctx:
        ids = scenes.upload(ctx, spec)
        stream = torch.cuda.Stream()
        out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
        x0 = spec.instances[0][1]
        for _ in range(warmup):
            ctx.raster_draw(ids, W, H, out, object_to_world=x0, stream=stream.cuda_stream)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(steps):
            ctx.raster_draw(ids, W, H, out, object_to_world=x0, stream=stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        ms = e0.elapsed_time(e1) / steps
    tris = sum(((v.shape[0] if i is None else len(i)) // 3) for v, i in spec.meshes)
    return {"config": f"{name} raster", "frame_ms": round(wall / steps * 1e3, 4), "gpu_ms": round(ms, 4),
            "triangles": int(tris), "resolution": f"{W}x{H}"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        a.gpus = world if world > 1 else a.gpus
    distributed = world > 1
    strips = distributed and a.assemble  # one frame split over ranks + RCCL gather
    torch.cuda.set_device(local)
    if distributed:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    spec = scenes.config(a.config)
    W, H = spec.width, spec.height
    ctx = rt.Context(local)
    scenes.upload(ctx, spec)
    ctx.set_schedule(rt.RT_SCHED_LANE if a.schedule == "lane" else rt.RT_SCHED_PACKET)
    binfo = [ctx.blas_info(b) for b in range(len(spec.meshes))]
    tinfo = ctx.tlas_info()

    rows = D.rank_rows(H, world, rank) if strips else None
    nrows = H if rows is None else len(rows)
    rows_per_rank = D.padded_rows(H, world) if strips else H
    stream = torch.cuda.Stream()
    sp = stream.cuda_stream
    local8 = torch.zeros((rows_per_rank, W, 4), dtype=torch.uint8, device="cuda")
    gathered = torch.zeros((world, rows_per_rank, W, 4), dtype=torch.uint8, device="cuda") if strips and rank == 0 else None
    frame = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") if strips and rank == 0 else None

    def step():
        ctx.dispatch(W, H, local8, None, rows=rows, stream=sp)
        if strips:
            with torch.cuda.stream(stream):
                D.gather_strips(local8, world, rank, gathered)
                if rank == 0:
                    ctx.assemble_strips(W, H, world, STRIP_ROWS, gathered, frame, stream=sp)

    # untimed counter pass: rays, box and triangle tests of this rank's share of the frame
    ctx.set_stats(True)
    ctx.stats_reset()
    ctx.dispatch(W, H, local8, None, rows=rows, stream=sp)
    torch.cuda.synchronize()
    st = ctx.stats()
    ctx.set_stats(False)
    rays_local = st["primary_rays"] + st["shadow_rays"]
    counts = torch.tensor([rays_local, st["primary_rays"], st["shadow_rays"]], dtype=torch.float64, device="cuda")
    if distributed:
        dist.all_reduce(counts)
    rays_step = int(counts[0].item())  # frames mode: N frames; strips mode: one frame

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()

    # one HIP event pair on the launch stream brackets the timed region: per-launch events would
    # put a timestamp (and its wait-for-idle) between back-to-back frames
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for k in range(a.steps):
        ctx.dispatch(W, H, local8, None, rows=rows, stream=sp)
        if strips:
            with torch.cuda.stream(stream):
                D.gather_strips(local8, world, rank, gathered)
                if rank == 0:
                    ctx.assemble_strips(W, H, world, STRIP_ROWS, gathered, frame, stream=sp)
    e1.record(stream)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # average launch duration over the timed region (strips mode: frame + gather + assembly)
    kernel_ms = e0.elapsed_time(e1) / a.steps
    tmax = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if distributed:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    tmax = float(tmax.item())

    if a.save_image and rank == 0:
        img = (frame if strips else local8[:H]).cpu().numpy()
        np.save(a.save_image, img)

    if rank == 0:
        value = rays_step * a.steps / tmax / 1e6
        bytes_launch = (BYTES_PER_AABB_TEST * st["aabb_tests"] + BYTES_PER_TRI_TEST * st["tri_tests"]
                        + BYTES_PER_PIXEL * W * nrows)
        achieved = bytes_launch / (kernel_ms * 1e-3) / 1e9
        traffic = load_traffic(a.config) if not strips else None
        cpu = None
        if not distributed and not a.no_cpu_baseline:
            cpu = cpu_baseline(spec, a.cpu_seconds)
        extra = []
        if not distributed and a.extra:
            sched = rt.RT_SCHED_LANE if a.schedule == "lane" else rt.RT_SCHED_PACKET
            for name in a.extra.split(","):
                extra.append(measure_config(name, max(5, a.steps // 2), 2, sched))
            extra.append(measure_raster("REF", max(5, a.steps // 2), 2))
        out = {
            "metric": "Mrays/sec (primary+shadow) at 1080p",
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(tmax / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if strips else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic camera/lights of BASELINE config; meshes teapot.obj/rabbit.obj from the reference",
            "config": {"workload": f"{spec.name}: {spec.model}.obj x{len(spec.instances) - 1} + plane, "
                                   f"{len(spec.lights)} light(s), {W}x{H}, {spec.spp} spp, shade "
                                   f"{['ref', 'lambert_shadow', 'primary'][spec.mode]}",
                       "rays_per_step": rays_step,
                       "rays_per_frame": rays_step if strips else int(rays_local),
                       "primary_rays": int(counts[1].item()), "shadow_rays": int(counts[2].item()), "parallelism": (f"strips{world}+gather" if strips else f"frames{world}"),
                       "schedule": a.schedule},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": "k_trace_frame" if a.schedule == "lane" else "k_trace_frame_packet", "kernel_ms": round(kernel_ms, 4),
                         "bytes_per_launch": int(bytes_launch),
                         "aabb_tests": int(st["aabb_tests"]), "tri_tests": int(st["tri_tests"]),
                         # the BVH (~1 MB) is L2-resident: algorithmic bytes are served by L2/L1, so
                         # frac vs HBM can exceed 1; the L2 roof (MI355X_MICROARCH.md) is the cache bound
                         "l2_peak": L2_PEAK_GBS, "l2_frac": round(achieved / L2_PEAK_GBS, 4)},
            "cpu_baseline": cpu,
            "build_ms": {"blas": [round(b.build_ms, 3) for b in binfo], "tlas": round(tinfo.build_ms, 3)},
            "extra": extra,
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
