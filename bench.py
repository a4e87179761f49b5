#!/usr/bin/env python3
"""Headline benchmark: Mrays/s (primary + shadow) at 1080p on MI355X — BASELINE.json config C2
(teapot.obj, 1 light, 1920x1080, primary + shadow rays) by default.

A step is one frame: RayGen -> TLAS/BLAS traversal -> shading + shadow rays -> RGBA8 (the
reference's DispatchRays, D3D12HelloTriangle.cpp:558-592). The scene is static: the LBVH build
runs once before the timed region and is reported separately (build_ms).

Multi-GPU (north star "frames are tiled across GPUs with an RCCL gather"): with
N > 1 a step is ONE frame split into interleaved 8-row strips (strip s -> rank s mod N): total work
fixed, "scaling": "strong". The loop is the library's own (rt_comm_* / rt_render_strips_frames behind
the C-ABI, csrc/rt_comm.cpp): each rank renders its strips as RGB8 into a pipeline slot on one of the
communicator's render streams, --frames-per-gather consecutive frames share a slot and ONE ncclGather
into rank 0 (--frames-per-launch of them rendered by one launch), and rank 0 assembles the RGBA8 frames
back on the slot's stream; gathers of one slot overlap the renders of the next. The frame latency
(enqueue -> frame assembled on rank 0, gather included) is timed after the timed region with
one frame per gather, one frame at a time (config.frame_latency_ms). `bench.py --gpus N` without
torchrun re-launches itself under torch.distributed.run (N processes, one per GPU) before anything
touches the GPU. The multi-GPU configs C4 (rabbit x64, 2 lights) and C5 (rabbit x256, 4 lights,
4K, 4 spp) are timed the same way at the same N and reported under "extra". When RCCL cannot be
used, the ranks fall back to a torch.distributed gather loop (config.strips_loop names the loop).
--loopback N (rehearsal, world 1): the library's loopback transport emulates N ranks on one GPU.

Frames in flight: consecutive frames are issued round robin over S render streams, each frame into
its own buffer slot, so the waves of frame k + 1 fill the wave slots the tail of frame k leaves
idle (a frame lasts as long as its slowest 8 x 8 tile; a reference-style renderer keeps two back
buffers for the same reason). Every frame is rendered in full; S (1..4) is picked by an untimed
autotune (pick_in_flight, per rank) and reported as config.frames_in_flight beside the one-stream frame time
(config.frame_ms_one_stream, the roofline's per-launch time). --in-flight 1 gives the serial loop.

value = rays traced in one step (all ranks, counted by the device counters in an untimed pass)
x steps / max-over-ranks wall time of the timed region.

The other configs under "extra" are timed over max(50, steps / 4) frames (multi-sample C5: max(10,
steps / 20)): with the driver's 20 steps a quarter of them was 5 frames, 0.07 ms of C1, where the host's issue and
the synchronise return dominated (the driver's BENCH_r03.json read C1 17.0 and C2F 67.2 Grays/s against 31.4 /
88.3 over 50 frames).

Tile balance (rt_set_tile_balance, the library's default): off while frames are in flight (the next frame fills
the slots the slowest tiles leave idle), on for the one-stream frame time and a rank's share when frames run one
at a time; config.tile_balance reports the last shape's plans.

Untimed before the W warmup frames: a clock settle (--settle-ms of frames: the GPU needs ~20 ms of
load to reach its steady clock; with 5 warmup frames alone the same build read 0.20 ms instead of
0.15 ms per frame; the ranks agree on its length), the tile-rows and frames-in-flight autotunes,
the counter pass, and a re-settle (--resettle-ms of frames on the timed loop's own streams and
buffers, renders only).
"""
from __future__ import annotations

import argparse
import hashlib
import importlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
L2_PEAK_GBS = 34500.0  # aggregate L2 bandwidth, 8 XCDs (MI355X_MICROARCH.md, L2 section)
# Bytes FETCHED per record visit (the roofline numerator; rt_api.h RT_STAT_*_FETCHES): the packet
# schedule loads each record once per wave into SGPRs, the per-lane schedule once per lane.
BYTES_PER_NODE_FETCH = 128  # one BVH4 node = one 128-B line (6 plane rows + child record)
BYTES_PER_TRI_FETCH = 48    # v0 / e1 / e2 rows of a TriRec
BYTES_PER_INST_FETCH = 64   # world-to-object 3x4 + translate flag + pool root of an InstanceRec
BYTES_PER_SHADE = 108       # per primary ray (upper bound: misses fetch nothing): 60 B of the
                            # instance's shading fields + 12 B indices + 36 B of 3 normals / positions
BYTES_PER_PIXEL = 4         # RGBA8 write
STRIP_ROWS = 8


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=100)
    p.add_argument("--settle-ms", type=float, default=300.0,
                   help="untimed frames before the warmup until this much GPU time has passed (clock ramp)")
    p.add_argument("--resettle-ms", type=float, default=30.0,
                   help="untimed frames on the timed loop's own streams right before the warmup (after the autotunes "
                        "and the counter pass)")
    p.add_argument("--config", default="C2")
    p.add_argument("--size", default="", help="WxH override (tests)")
    p.add_argument("--schedule", default="packet", choices=["packet", "lane"])
    p.add_argument("--mode", default="auto", choices=["auto", "strips", "frames"],
                   help="N>1: strips = one frame tiled over ranks + RCCL gather (default); frames = N "
                        "independent replicas (no collective)")
    p.add_argument("--no-pipeline", action="store_true", help="strips: gather after each frame, no overlap")
    p.add_argument("--phase-frames", type=int, default=64,
                   help="strips through the native loop: frames of the per-phase pass after the timed region "
                        "(config.phases; 0: none)")
    p.add_argument("--frames-per-gather", type=int, default=4,
                   help="strips through the native loop: consecutive frames whose strips one ncclGather moves "
                        "(rt_comm_set_batch; the gather half of a step is paid once per this many frames)")
    p.add_argument("--frames-per-launch", type=int, default=0,
                   help="strips through the native loop: frames rendered by one launch per rank "
                        "(rt_render_strips_frames); 0 = --frames-per-gather")
    p.add_argument("--loopback", type=int, default=0,
                   help="rehearsal at world 1 (tests): the native strips loop over the library's loopback transport "
                        "emulating this many ranks on one GPU (rt_comm_init_loopback)")
    p.add_argument("--latency-frames", type=int, default=20,
                   help="strips: single frames timed enqueue -> assembled on rank 0 (config.frame_latency_ms)")
    p.add_argument("--in-flight", type=int, default=0,
                   help="frames in flight (render streams, one buffer each); 0 = untimed autotune over 1..4")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="minimum wall time of the CPU baseline sample")
    p.add_argument("--save-image", default="", help="write the rank-0 frame as .npy")
    p.add_argument("--extra", default=None,
                   help="comma list of further configs ('' to skip); default N=1: C1,C2F,C3,C4,C5,REF (+ REF "
                        "raster); N>1: C4,C5 tiled over the same ranks")
    return p.parse_args(argv)


# ---------------------------------------------------------------------------------------------
# launcher: one process per GPU
# ---------------------------------------------------------------------------------------------

class stdout_to_stderr:
    """RCCL prints a version banner to stdout when a communicator is created (with NCCL_DEBUG set): while one is
    created, fd 1 points at stderr (C stdio flushed on both edges), so rank 0's stdout stays the one JSON line."""

    def __enter__(self):
        import ctypes
        self._libc = ctypes.CDLL(None)
        sys.stdout.flush()
        self._libc.fflush(None)
        self._saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        sys.stdout.flush()
        self._libc.fflush(None)
        os.dup2(self._saved, 1)
        os.close(self._saved)
        return False


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn(a, argv) -> int:
    """`bench.py --gpus N` outside torchrun: run N ranks under torch.distributed.run as a CHILD
    process (nothing here has touched the GPU) and return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


# ---------------------------------------------------------------------------------------------
# backends: the HIP library (product) or a test renderer (tests/, CPU + gloo)
# ---------------------------------------------------------------------------------------------

class HipBackend:
    """rt_* through the C-ABI on this rank's GPU; collectives over RCCL."""
    dist_backend = "nccl"
    multi_stream = True  # streams run concurrently: frames in flight are worth measuring

    def __init__(self, local: int):
        import realtimeraytracing_gradproject_amd as rt
        self.rt = rt
        # RT_BENCH_ONE_DEVICE=1 (rehearsal only): every rank on device 0, to exercise the RCCL path on a
        # one-GPU box; never used for a reported number
        if os.environ.get("RT_BENCH_ONE_DEVICE") == "1":
            local = 0
        torch.cuda.set_device(local)
        self.local = local
        self.device = torch.device("cuda", local)
        self.ctx = None

    def init_pg(self):
        if os.environ.get("RT_BENCH_ONE_DEVICE") == "1":  # rehearsal: RCCL refuses two ranks on one GPU
            dist.init_process_group("gloo")
            return
        with stdout_to_stderr():
            dist.init_process_group("nccl", device_id=self.device)
            dist.barrier()  # the process group's communicator is created here (eagerly, not in the timed loop)

    def load(self, spec, schedule: str):
        from realtimeraytracing_gradproject_amd import scenes
        if self.ctx is not None:
            self.ctx.close()
        self.ctx = self.rt.Context(self.local)
        scenes.upload(self.ctx, spec)
        self.ctx.set_schedule(self.rt.RT_SCHED_LANE if schedule == "lane" else self.rt.RT_SCHED_PACKET)
        self.spec = spec
        first = ([round(self.ctx.blas_info(b).build_ms, 4) for b in range(len(spec.meshes))],
                 round(self.ctx.tlas_info().build_ms, 4))
        # warm rebuilds (a hot reload, D3D12HelloTriangle.cpp:1482-1568): the first build above also
        # pays the kernels' first launch
        blas_w, tlas_w = [[] for _ in spec.meshes], []
        for _ in range(5):
            for b, (v, i) in enumerate(spec.meshes):
                self.ctx.blas_rebuild(b, v, i)
                blas_w[b].append(self.ctx.blas_info(b).build_ms)
            self.ctx.tlas_build([(m, x, iid, hg) for (m, x, iid, hg) in spec.instances])
            tlas_w.append(self.ctx.tlas_info().build_ms)
        med = lambda xs: round(sorted(xs)[len(xs) // 2], 4)  # noqa: E731
        # per-frame TLAS update (TopLevelASGenerator.cpp:202-222 from OnUpdate, D3D12HelloTriangle.cpp:421-433):
        # the host wall time of rt_tlas_build(update_only) (double-buffered, no device-wide sync) and its kernels
        upd_wall, upd_dev = [], []
        inst = [(m, x, iid, hg) for (m, x, iid, hg) in spec.instances]
        for _ in range(10):
            self.ctx.tlas_build(inst, update_only=True)
            upd_wall.append(self.ctx.tlas_build_wall_ms())
            upd_dev.append(self.ctx.tlas_info().build_ms)
        return first + ([med(x) for x in blas_w], med(tlas_w), med(upd_wall), med(upd_dev))

    def zeros(self, shape):
        return torch.zeros(shape, dtype=torch.uint8, device=self.device)

    def stream(self):
        return torch.cuda.Stream(device=self.device)

    def event(self, timing=False):
        return torch.cuda.Event(enable_timing=timing)

    def use_stream(self, s):
        return torch.cuda.stream(s)

    def set_tile_rows(self, rows: int):
        self.ctx.set_tile_rows(rows)

    def tile_balance(self) -> dict:
        return self.ctx.tile_balance_info()

    def sync_event(self):
        """Render/gather hand-off of the strips loop: rt_event_* (no timestamp, no system-scope
        fence: ~3 us less per record than a torch.cuda.Event on the frame's critical path)."""
        ev = self.rt.PipelineEvent()
        ev.recorded = False
        return ev

    def record(self, ev, stream):
        ev.record(stream.cuda_stream)
        ev.recorded = True

    def wait(self, stream, ev):
        if ev.recorded:
            ev.wait_on(stream.cuda_stream)

    def synchronize(self):
        torch.cuda.synchronize(self.device)

    def dispatch(self, buf, rows, stream):
        self.ctx.dispatch(self.spec.width, self.spec.height, buf, None, rows=rows, stream=stream.cuda_stream)

    def counted(self, buf, rows, stream) -> dict:
        self.ctx.set_stats(True)
        self.ctx.stats_reset()
        self.dispatch(buf, rows, stream)
        self.synchronize()
        st = self.ctx.stats()
        self.ctx.set_stats(False)
        return st

    def assemble(self, world, gathered, frame, stream):
        self.ctx.assemble_strips(self.spec.width, self.spec.height, world, STRIP_ROWS, gathered, frame,
                                 stream=stream.cuda_stream)

    def raster(self, spec, steps, warmup):
        return measure_raster(self, spec, steps, warmup)

    @property
    def native_strips(self) -> bool:
        """Strips mode through the C-ABI's own frame loop (rt_render_strips: render -> ncclGather -> assembly
        issued from C++); the gloo rehearsal on one device keeps the torch.distributed loop."""
        return os.environ.get("RT_BENCH_ONE_DEVICE") != "1" and os.environ.get("RT_BENCH_TORCH_STRIPS") != "1"

    def comm_open(self, world: int, rank: int, loopback: int = 0):
        """rt_comm over this rank's context: rank 0's ncclUniqueId is broadcast over the torch process group.
        loopback N (world 1): the library's loopback transport emulating N ranks on this GPU."""
        if loopback:
            return self.rt.Comm.loopback(self.ctx, loopback)
        with stdout_to_stderr():
            uid = self.rt.comm_unique_id() if rank == 0 else bytes(self.rt.RT_COMM_ID_BYTES)
            t = torch.tensor(list(uid), dtype=torch.uint8, device=self.device)
            dist.broadcast(t, 0)
            return self.rt.Comm(self.ctx, world, rank, bytes(t.cpu().tolist()))

    def render_strips(self, comm, frames, stream):
        """len(frames) frames in one rt_render_strips_frames call (one launch per rank)."""
        s = stream.cuda_stream if stream is not None else None
        if len(frames) == 1:
            comm.render_strips(self.spec.width, self.spec.height, frames[0], s, STRIP_ROWS)
        else:
            comm.render_strips_frames(self.spec.width, self.spec.height, frames, None, s, STRIP_ROWS)

    def close(self):
        if self.ctx is not None:
            self.ctx.close()
            self.ctx = None


def make_backend(local: int):
    """RT_BENCH_TEST_BACKEND=module:factory (tests only) swaps in a CPU renderer with gloo so the
    launcher, partition, gather, assembly and timing code below runs without a GPU."""
    hook = os.environ.get("RT_BENCH_TEST_BACKEND", "")
    if hook:
        mod, _, fn = hook.partition(":")
        return getattr(importlib.import_module(mod), fn)(local)
    return HipBackend(local)


# ---------------------------------------------------------------------------------------------
# the measured loop
# ---------------------------------------------------------------------------------------------

def strip_plan(H: int, world: int, rank: int):
    from realtimeraytracing_gradproject_amd import distributed as D
    return D.rank_rows(H, world, rank), D.padded_rows(H, world)


def pick_tile_rows(be, buf, rows, stream, frames: int = 8, rounds: int = 3):
    """Untimed autotune of rt_set_tile_rows: this rank's render alone at 8 x 8 and 8 x 4 pixel tiles per
    wave, alternating, best of `rounds`; keeps the faster (the image is the same). 8 x 4 wins only when
    so few waves run that the slowest tile sets the frame time (one rank's strips of a frame tiled over
    many GPUs); a backend without the setting keeps 8. Returns (rows, {rows: ms per frame})."""
    if not hasattr(be, "set_tile_rows"):
        return 8, None
    best = {8: float("inf"), 4: float("inf")}
    for _ in range(rounds):
        for tr in (8, 4):
            be.set_tile_rows(tr)
            be.dispatch(buf, rows, stream)
            e0, e1 = be.event(True), be.event(True)
            e0.record(stream)
            for _ in range(frames):
                be.dispatch(buf, rows, stream)
            e1.record(stream)
            be.synchronize()
            best[tr] = min(best[tr], e0.elapsed_time(e1) / frames)
    pick = 4 if best[4] < best[8] else 8
    be.set_tile_rows(pick)
    return pick, {k: round(v, 4) for k, v in best.items()}


def pick_in_flight(be, W, NR, rows, frames: int = 16, rounds: int = 3, choices=(1, 2, 3, 4)):
    """Untimed autotune of the frames in flight: `frames` renders of this rank's share issued round
    robin over the first S streams of one stream pool into S buffers, S in `choices`, interleaved,
    best of `rounds` (host wall clock around the synchronised loop); the largest S within 1 % of the fastest. With S > 1 the waves of frame
    k + 1 fill the wave slots the tail of frame k leaves idle (a frame ends with its slowest 8 x 8
    tile; tools/overlap_probe.py). Which streams share a hardware queue is the HIP runtime's choice
    (two streams can land on one queue and then run one after the other), so the count is
    measured, not assumed, and the caller renders on the very streams that were measured. A backend
    without streams of its own keeps 1. Returns (S, {S: ms per frame}, the S streams)."""
    if not getattr(be, "multi_stream", False):
        return 1, None, None
    pool = [be.stream() for _ in range(max(choices))]
    bufs = [be.zeros((NR, W, 4)) for _ in range(max(choices))]
    best = {n: float("inf") for n in choices}
    for _ in range(rounds):
        for n in choices:
            be.synchronize()
            t0 = time.perf_counter()
            for k in range(frames):
                be.dispatch(bufs[k % n], rows, pool[k % n])
            be.synchronize()
            best[n] = min(best[n], (time.perf_counter() - t0) * 1e3 / frames)
    # near-ties (within 1 %, the measurement's noise) go to the most frames in flight: in a short timed region
    # (the driver's 20 frames) two streams run their frames in lockstep pairs, three or four keep the SIMDs fuller
    # (profiles/r03_short_region_probe.txt, tools/short_inflight.sh)
    fastest = min(best.values())
    pick = max(n for n in choices if best[n] <= fastest * 1.01)
    return pick, {n: round(v, 4) for n, v in best.items()}, pool[:pick]


def run_config(*args, **kw):
    """Builds the scene, counts one step's rays (untimed), settles, warms up, then times exactly
    `steps` steps between barrier + synchronize on both sides. Returns a dict (rank 0 meaningful).
    in_flight: frames in flight (render streams, each with its own buffer slot); 0 = autotune.
    The failure path: an exception while the native communicator is open aborts it (rt_comm_abort: no draining
    collective that the other ranks, out of step after the error, might never match) before it propagates."""
    held = {}
    try:
        return _run_config(*args, held=held, **kw)
    except BaseException:
        if held.get("comm") is not None:
            held.pop("comm").abort()
        raise


def _run_config(be, spec, world: int, rank: int, steps: int, warmup: int, settle_ms: float, strips: bool,
                pipeline: bool, schedule: str, save_image: str = "", in_flight: int = 0, resettle_ms: float = 0.0,
                frames_per_gather: int = 1, frames_per_launch: int = 0, loopback: int = 0, latency_frames: int = 20,
                phase_frames: int = 0, held: dict = None):
    from realtimeraytracing_gradproject_amd import distributed as D
    distributed = world > 1
    W, H = spec.width, spec.height
    build = be.load(spec, schedule)
    if strips and loopback:  # one process renders every emulated rank's strips: time and count the whole frame
        rows, rows_per_rank = None, H
    elif strips:
        rows, rows_per_rank = strip_plan(H, world, rank)
    else:
        rows, rows_per_rank = None, H
    NR = rows_per_rank
    comm = be.stream() if strips else None

    def settle(ms, bufs, streams):
        """Untimed frames on `streams` (round robin into `bufs`) until `ms` of wall time has passed; the ranks
        agree on the length (every 4 frames an all-reduce MAX of "still settling"), so no collective is left
        unmatched. Renders only: no gather."""
        t0 = time.perf_counter()
        n = 0
        while True:
            for _ in range(4):
                be.dispatch(bufs[n % len(bufs)], rows, streams[n % len(streams)])
                n += 1
            be.synchronize()
            more = torch.tensor([1.0 if (time.perf_counter() - t0) * 1e3 < ms else 0.0],
                                dtype=torch.float64, device=be.device)
            if distributed:
                dist.all_reduce(more, op=dist.ReduceOp.MAX)
            if more.item() == 0.0:
                break

    # clock settle (untimed) on a plain single-stream loop before any autotune
    if settle_ms > 0:
        probe_b = be.zeros((NR, W, 4))
        settle(settle_ms, [probe_b], [be.stream()])
        del probe_b

    tile_rows, tile_ms = pick_tile_rows(be, be.zeros((NR, W, 4)), rows, be.stream())
    measured = None
    if in_flight > 0:
        nstream, flight_ms = in_flight, None
    else:
        nstream, flight_ms, measured = pick_in_flight(be, W, NR, rows)
    render = measured if measured else [be.stream() for _ in range(nstream)]
    native = strips and getattr(be, "native_strips", False)
    if native and not loopback:  # every rank agrees before the collective rt_comm_init (no RCCL: the torch loop)
        ok = torch.tensor([1.0 if be.rt.comm_available() else 0.0], dtype=torch.float64, device=be.device)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        native = ok.item() == 1.0
    rcomm = None
    if native:  # a communicator that fails to come up on any rank sends every rank to the torch.distributed loop
        try:
            rcomm = be.comm_open(world, rank, loopback) if loopback else be.comm_open(world, rank)
            held["comm"] = rcomm
        except Exception as ex:  # noqa: BLE001  (RtError from rt_comm_init: reported, then the fallback)
            print(f"bench: rt_comm_init failed on rank {rank} ({ex}); using the torch.distributed strips loop",
                  file=sys.stderr, flush=True)
        up = torch.tensor([1.0 if rcomm is not None else 0.0], dtype=torch.float64, device=be.device)
        dist.all_reduce(up, op=dist.ReduceOp.MIN)
        if up.item() != 1.0:
            if rcomm is not None:  # another rank has no communicator: no collective may be issued on this one
                held.pop("comm").abort()
            rcomm, native = None, False
        elif frames_per_gather > 1:  # the same on every rank (it sizes the collective); the library takes 1 .. 4
            rcomm.set_batch(min(frames_per_gather, 4))
    nslot = max(nstream, 2 if (strips and pipeline) else 1)
    local = [be.zeros((rows_per_rank, W, 4)) for _ in range(nslot)]
    gathered = ([be.zeros((world, rows_per_rank, W, 4)) if rank == 0 else None for _ in range(nslot)]
                if strips and not native else None)
    frame = ([be.zeros((H, W, 4)) if rank == 0 else None for _ in range(rcomm.depth if native else nslot)]
             if strips else None)
    rendered = [be.sync_event() for _ in range(nslot)]
    freed = [be.sync_event() for _ in range(nslot)]
    parts = [D.gather_parts(gathered[s], world, rank) for s in range(nslot)] if strips and not native else None

    ncall = [0]
    fpl = max(1, min(frames_per_launch or (rcomm.batch if rcomm is not None else 1), 4))
    if rcomm is not None:
        fpl = min(fpl, rcomm.batch)

    def issue_native(n: int, per_call: int):
        """n frames through rt_render_strips_frames, `per_call` per call (one launch per call on this rank): render
        on a slot's stream, ncclGather on the communicator's gather stream, rank 0's assembly back on the slot's
        stream, the slot pipeline and its events inside the library. Frame buffer i serves the i-th frame mod the
        pipeline depth."""
        # frames in flight: the communicator's own three render streams (NULL), which sit on hardware queues of
        # their own, apart from the gathers' (DESIGN §7); one frame at a time: this rank's stream
        rs = render[0] if nstream == 1 else None
        while n > 0:
            m = min(n, per_call)
            bufs = [frame[(ncall[0] + j) % rcomm.depth] if rank == 0 else None for j in range(m)]
            ncall[0] += m
            be.render_strips(rcomm, bufs, rs)
            n -= m

    def step_native(k: int):
        issue_native(1, 1)

    def step(k: int):
        """One frame. In strips mode the caller holds `comm` as the current stream (the gather runs
        on it; everything else names its stream explicitly), so no stream context is entered per step."""
        s = k % nslot
        rs = render[s % nstream]  # a slot always renders on the same stream: its reuse is stream-ordered
        if strips:
            be.wait(rs, freed[s])  # slot s free: the gather of frame k - nslot is done
        be.dispatch(local[s], rows, rs)
        if strips:
            be.record(rendered[s], rs)
            be.wait(comm, rendered[s])
            D.gather_strips(local[s], world, rank, gathered[s], parts=parts[s])
            if rank == 0:
                be.assemble(world, gathered[s], frame[s], comm)
            be.record(freed[s], comm)

    import contextlib
    on_comm = (lambda: be.use_stream(comm)) if strips and not native else contextlib.nullcontext
    if native:
        step = step_native  # noqa: F811

    k = 0
    # untimed counter pass: rays, tests and record fetches of this rank's share of one step
    st = be.counted(local[0], rows, render[0])
    counts = torch.tensor([st["primary_rays"] + st["shadow_rays"], st["primary_rays"], st["shadow_rays"]],
                          dtype=torch.float64, device=be.device)
    if distributed:
        dist.all_reduce(counts)
    rays_step = int(counts[0].item())  # strips: one frame over all ranks; frames mode: N frames

    def drain():
        """Everything issued so far has finished: with the native loop the library's issue thread first
        enqueues the gathers it was handed (rt_comm_synchronize), then the device drains."""
        if rcomm is not None:
            rcomm.synchronize()
        be.synchronize()

    # re-settle (untimed): the autotunes and the counter pass leave the GPU between loads; frames on the very
    # streams and buffers of the timed loop bring it back to its steady state before the warmup
    if resettle_ms > 0:
        settle(resettle_ms, local, render)

    # warmup (untimed)
    with on_comm():
        if native:
            issue_native(warmup, fpl)
            k += warmup
        else:
            for _ in range(warmup):
                step(k)
                k += 1
    drain()
    if distributed:
        dist.barrier()
    be.synchronize()

    # timed region (wall clock, synchronised on both sides). With one render stream and no strips a
    # HIP event pair on it also gives the per-launch kernel time (per-launch events would put a
    # timestamp between back-to-back frames)
    single = nstream == 1 and not strips
    e0, e1 = be.event(True), be.event(True)
    t0 = time.perf_counter()
    e0.record(render[0])
    with on_comm():
        if native:
            issue_native(steps, fpl)
            k += steps
        else:
            for _ in range(steps):
                step(k)
                k += 1
    e1.record(render[0])
    drain()
    if distributed:
        dist.barrier()
    be.synchronize()
    elapsed = time.perf_counter() - t0
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=be.device)
    if distributed:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    tmax = float(tmax.item())
    render_ms = e0.elapsed_time(e1) / steps

    if not single:
        # the roofline's kernel time: this rank's render alone, back to back on one stream (untimed
        # for value)
        be.synchronize()
        f0, f1 = be.event(True), be.event(True)
        f0.record(render[0])
        for _ in range(max(5, min(steps, 50))):
            be.dispatch(local[0], rows, render[0])
        f1.record(render[0])
        be.synchronize()
        kernel_ms = f0.elapsed_time(f1) / max(5, min(steps, 50))
    else:
        kernel_ms = render_ms

    # frame latency (dispatch enqueue -> the RGBA8 frame complete on the root GPU, the RCCL gather
    # included; the reference's frame time spans submit -> fence, D3D12HelloTriangle.cpp:436-470): strips mode, one
    # frame per gather, one frame at a time, host clock from the call to the synchronised drain; rank 0's median
    latency_ms = None
    fpg = rcomm.batch if rcomm is not None else None  # the timed loop's (the latency pass below gathers 1 frame)
    if strips and latency_frames > 0:
        if rcomm is not None:
            rcomm.set_batch(1)
        lat = []
        with on_comm():
            for _ in range(latency_frames):
                if distributed:
                    dist.barrier()
                t1 = time.perf_counter()
                if native:
                    issue_native(1, 1)
                else:
                    step(k)
                    k += 1
                drain()
                lat.append(time.perf_counter() - t1)
        latency_ms = float(np.median(lat)) * 1e3

    # per-phase cost of a step (the N > 1 line names its own binding cost), untimed for `value`: the
    # timed loop's batching and streams again, with the communicator's timing-event pairs around each render, gather
    # and assembly (rt_comm_set_phase_timing), over the wall clock of the pass
    phases = None
    if native and phase_frames > 0:
        rcomm.set_batch(fpg)
        rcomm.set_phase_timing(True)
        if distributed:
            dist.barrier()
        be.synchronize()
        t1 = time.perf_counter()
        issue_native(phase_frames, fpl)
        ps = rcomm.phase_stats()  # drains the pipeline
        be.synchronize()
        wall = time.perf_counter() - t1
        rcomm.set_phase_timing(False)
        phases = phase_summary(ps, wall, world, rank, loopback, distributed, be.device)

    if save_image and rank == 0:
        last = (ncall[0] - 1) % rcomm.depth if native else (k - 1) % nslot
        if native:
            rcomm.synchronize()
        img = frame[last] if strips else local[last][:H]
        np.save(save_image, img.cpu().numpy())
    if rcomm is not None:
        rcomm.close()
        held.pop("comm", None)
    # the tile balance of this rank's last launch shape (rt_tile_balance_info: plans run, tiles split, ...)
    tb = be.tile_balance() if hasattr(be, "tile_balance") else None
    return {"rays_step": rays_step, "primary": int(counts[1].item()), "shadow": int(counts[2].item()), "fpg": fpg,
            "fpl": fpl if native else None, "latency_ms": latency_ms, "loopback": loopback if native else 0,
            "phases": phases,
            "tile_balance": tb,
            "tmax": tmax, "kernel_ms": kernel_ms, "stats": st, "build": build, "rows_local": len(rows) if rows is not None else H,
            "tile_rows": tile_rows, "tile_ms": tile_ms, "in_flight": nstream, "in_flight_ms": flight_ms,
            "strips_loop": ("rt_render_strips_frames (C-ABI: render RGB8 strips -> "
                            + (f"loopback gather of {loopback} emulated ranks" if loopback else "ncclGather")
                            + " -> RGBA8 assembly; "
                            + ("the communicator's 3 render streams)" if nstream > 1 else "one render stream)")
                            if native else
                            "torch.distributed gather" if strips else None)}


# ---------------------------------------------------------------------------------------------
# roofline
# ---------------------------------------------------------------------------------------------

def phase_summary(ps: dict, wall_s: float, world: int, rank: int, loopback: int, distributed: bool, device) -> dict:
    """Per-frame phases of the native strips loop on this rank (rank 0's line): the render of its share (loopback:
    every emulated rank's share, one GPU renders them all), the gather (gather stream, from this rank's render done to
    the gather's end: the transfer plus any wait for the other ranks), rank 0's assembly, the host's issue (caller
    thread per frame, the library's issue thread per frame), the bytes into rank 0 and their rate over the gather
    time, the pass's period; the render share's max / min over the ranks (all-reduce)."""
    f = max(ps["frames"], 1.0)
    render = ps["render_ms"] / f
    rr = torch.tensor([render, -render], dtype=torch.float64, device=device)
    if distributed:
        dist.all_reduce(rr, op=dist.ReduceOp.MAX)
    period = wall_s * 1e3 / f
    gather = ps["gather_ms"] / f
    asm = ps["assembly_ms"] / f
    out = {"frames": int(ps["frames"]), "period_ms": round(period, 4),
           "render_share_ms": round(render, 4),
           "render_share_ms_max": round(float(rr[0].item()), 4), "render_share_ms_min": round(float(-rr[1].item()), 4),
           "render_launches_per_frame": round(ps["renders"] / f, 3),
           "gather_ms": round(gather, 4), "assembly_ms": round(asm, 4),
           "host_issue_us": round(ps["host_us"] / f, 2), "issue_thread_us": round(ps["issue_us"] / f, 2),
           "bytes_into_rank0_per_frame": int(ps["bytes_in"] / f),
           "ingress_GBps_over_gather": (round(ps["bytes_in"] / (ps["gather_ms"] * 1e-3) / 1e9, 3)
                                        if ps["gather_ms"] > 0 else None),
           "ingress_GBps_at_period": round(ps["bytes_in"] / f / (period * 1e-3) / 1e9, 3) if period > 0 else None,
           "phase_sum_over_period": round((render + gather + asm) / period, 3) if period > 0 else None,
           "rank": rank, "world": world, "loopback_ranks": loopback or None,
           "note": ("loopback: one GPU renders every emulated rank's share (render_share_ms is their sum) and the "
                    "gather is a device copy" if loopback else
                    "this rank's share; gather = ncclGather from this rank's render done to its end")}
    return out


def lib_sha() -> str:
    p = os.path.join(ROOT, "realtimeraytracing_gradproject_amd", "lib", "librtamd.so")
    try:
        with open(p, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
        return ""


def load_profile(config: str):
    """Per-launch HBM traffic and SQ issue counts of the trace kernel from the committed rocprofv3
    passes (profiles/roofline_inputs.json, written by tools/roofline.py summarize)."""
    try:
        with open(os.path.join(ROOT, "profiles", "roofline_inputs.json")) as f:
            return json.load(f).get(config)
    except (OSError, ValueError):
        return None


def fetched_bytes(st: dict, pixels: int) -> int:
    return (BYTES_PER_NODE_FETCH * st["node_fetches"] + BYTES_PER_TRI_FETCH * st["tri_fetches"]
            + BYTES_PER_INST_FETCH * st["instance_fetches"] + BYTES_PER_SHADE * st["primary_rays"]
            + BYTES_PER_PIXEL * pixels)


# SURVEY.md §8(d)'s per-lane algorithmic bytes: 24 B per AABB test + 36 B per triangle test + 4 B per pixel. The
# packet walk loads a node / triangle once per WAVE into SGPRs and every lane tests it from there, so this model
# counts a wave-uniform scalar fetch 64 times: a logical figure (it exceeds the HBM peak), not memory traffic.
LOGICAL_BYTES_PER_AABB_TEST = 24
LOGICAL_BYTES_PER_TRI_TEST = 36
N_CU, N_SIMD = 256, 1024


def logical_bytes(st: dict, pixels: int) -> int:
    return (LOGICAL_BYTES_PER_AABB_TEST * st["aabb_tests"] + LOGICAL_BYTES_PER_TRI_TEST * st["tri_tests"]
            + BYTES_PER_PIXEL * pixels)


def roofline(config: str, st: dict, pixels: int, kernel_ms: float, schedule: str) -> dict:
    """The trace kernel against every roof it could meet, and the binding one on top (the line's
    achieved / peak / frac are the BOUND pipe's, so frac = achieved / peak = fracs[bound]):
      l2    bytes fetched per launch (per-wave record fetches from the STATS pass) / kernel time vs the L2 roof;
      hbm   measured HBM bytes per launch (rocprofv3 PMC, profiles/) / kernel time vs 8 TB/s;
      valu  wave64 VALU instructions per launch / (1024 SIMDs x cycles / 2), from the committed SQ counters, stated
            as G instructions / s at the counters' shader clock (cycles per XCD / the profiled kernel time);
      salu  scalar instructions / (256 CUs x cycles), likewise.
    `logical_bytes` is SURVEY §8(d)'s per-lane model, labelled: it counts wave-uniform fetches once per lane."""
    b = fetched_bytes(st, pixels)
    l2_ach = b / (kernel_ms * 1e-3) / 1e9
    prof = load_profile(config) or {}
    traffic = prof.get("hbm_bytes_per_launch")
    issue = prof.get("issue")
    pipes = {"l2": {"achieved": round(l2_ach, 1), "peak": L2_PEAK_GBS, "unit": "GB/s", "frac": l2_ach / L2_PEAK_GBS,
                    "bytes_per_launch": int(b)}}
    if traffic:
        hb = traffic / (kernel_ms * 1e-3) / 1e9
        pipes["hbm"] = {"achieved": round(hb, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": hb / HBM_PEAK_GBS,
                        "source": prof.get("source")}
    rk = prof.get("rocprof_kernel_avg_ms")
    if issue and rk:
        cyc = issue["cycles_per_xcd"]
        clk = cyc / (rk * 1e6)  # GHz: the counters' cycles over the profiled kernel time
        for pipe, per_launch, width in (("valu", issue["valu_per_launch"], N_SIMD / 2),
                                        ("salu", issue["salu_per_launch"], N_CU)):
            frac = issue[pipe + "_frac"]
            pipes[pipe] = {"achieved": round(per_launch / (rk * 1e6), 2), "peak": round(width * clk, 2),
                           "unit": "G instructions/s", "frac": frac, "per_launch": per_launch,
                           "clock_ghz": round(clk, 3)}
    fracs = {k: v["frac"] for k, v in pipes.items()}
    bound = max(fracs, key=fracs.get)
    top = pipes[bound]
    lb = logical_bytes(st, pixels)
    out = {"bound": bound, "achieved": top["achieved"], "peak": top["peak"], "unit": top["unit"],
           "frac": round(top["frac"], 4), "traffic": traffic,
           "l2_frac": round(fracs["l2"], 4),
           "kernel": "k_trace_frame" if schedule == "lane" else "k_trace_frame_packet8",
           "kernel_ms": round(kernel_ms, 4), "bytes_per_launch": int(b),
           "model": (f"{BYTES_PER_NODE_FETCH} B/node fetch + {BYTES_PER_TRI_FETCH} B/triangle fetch + "
                     f"{BYTES_PER_INST_FETCH} B/instance fetch (per wave in packets) + {BYTES_PER_SHADE} B/primary "
                     f"ray shading + {BYTES_PER_PIXEL} B/pixel"),
           "logical_bytes": {"bytes_per_launch": int(lb), "GB_per_s": round(lb / (kernel_ms * 1e-3) / 1e9, 1),
                             "model": (f"SURVEY 8(d): {LOGICAL_BYTES_PER_AABB_TEST} B/AABB test + "
                                       f"{LOGICAL_BYTES_PER_TRI_TEST} B/triangle test (per lane) + "
                                       f"{BYTES_PER_PIXEL} B/pixel"),
                             "note": "per-lane logical bytes: a wave-uniform scalar fetch counted once per lane; "
                                     "not memory traffic (l2 / hbm are)"},
           "node_fetches": int(st["node_fetches"]), "tri_fetches": int(st["tri_fetches"]),
           "instance_fetches": int(st["instance_fetches"]),
           "aabb_tests": int(st["aabb_tests"]), "tri_tests": int(st["tri_tests"]),
           "fracs": {k: round(v, 4) for k, v in fracs.items()},
           "pipes": {k: {**v, "frac": round(v["frac"], 4)} for k, v in pipes.items()}}
    if traffic:
        out["hbm"] = {"achieved": pipes["hbm"]["achieved"], "peak": HBM_PEAK_GBS,
                      "frac": round(fracs["hbm"], 4), "source": prof.get("source")}
    if issue:
        out["issue"] = dict(issue)
        out["issue"]["profile_lib_sha"] = prof.get("lib_sha")
        out["issue"]["stale"] = bool(prof.get("lib_sha")) and prof.get("lib_sha") != lib_sha()
    return out


# ---------------------------------------------------------------------------------------------
# CPU baseline (rank 0, N = 1): the oracle's scalar per-ray traversal of the same BVH
# ---------------------------------------------------------------------------------------------

def _cgroup_cpus():
    """CPUs' worth of time the cgroup lets this process use (cpu.max quota / period), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        return None


def _frame_median(o, spec, threads: int, frames: int = 5):
    """BASELINE.md section 3 timing: one warm-up frame, then the median wall time of `frames` frames of the
    per-ray traversal (the CPU form: one traversal per ray, LANE order) at `threads` threads."""
    o.render_spec(spec, nthreads=threads, want_float=False, schedule=1)
    ts = []
    for _ in range(frames):
        t0 = time.perf_counter()
        o.render_spec(spec, nthreads=threads, want_float=False, schedule=1)
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), float(sum(ts))


def cpu_baseline(spec, seconds: float = 0.0):
    """BASELINE.md section 3's CPU baseline: oracle/libbaseline.so — the oracle's scalar C restatement
    (per-ray traversal of the identical trees, identical shading, pthreads over interleaved rows) built at
    -O3 with the counters compiled out (frames identical to the checker's) — on the same frame on this
    host. Threads: one per CPU the process may run on (os.sched_getaffinity) and, when a cgroup CPU quota
    caps the process below that (the GPU box gives one GPU's job 16 CPUs' worth of time on a 256-CPU host),
    one per CPU of the quota; `value` is the better. Plus one thread, the checker build (liboracle.so: -O2,
    counters on) for comparison, and C1 (BASELINE configs[0]: teapot 512^2 primary only). Rays per frame come
    from the checker's counters (deterministic). Each figure: one warm-up frame, median of 5 frames.
    `seconds` is unused (kept for the CLI)."""
    import math
    import oracle
    from realtimeraytracing_gradproject_amd import scenes

    ncpu = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = _cgroup_cpus()
    counts = [min(256, ncpu)]  # oracle_render caps its pool at 256 threads
    if quota and math.ceil(quota) < counts[0]:
        counts.append(max(1, math.ceil(quota)))
    blib = oracle.baseline_lib()
    t_all = time.perf_counter()

    def rays_of(sp):
        _, _, st = oracle.Scene(sp).render_spec(sp, nthreads=counts[-1], want_float=False, schedule=1)
        return int(st[0] + st[1])

    rays = rays_of(spec)
    o = oracle.Scene(spec, library=blib)
    runs = []
    for th in counts:
        med, wall = _frame_median(o, spec, th)
        runs.append({"threads": th, "value": round(rays / med / 1e6, 3), "frame_s": round(med, 4),
                     "wall_s": round(wall, 2)})
    best = max(runs, key=lambda r: r["value"])
    med1, _ = _frame_median(o, spec, 1)
    chk, _ = _frame_median(oracle.Scene(spec), spec, best["threads"], frames=3)
    c1 = scenes.config("C1")
    r1 = rays_of(c1)
    o1 = oracle.Scene(c1, library=blib)
    m1, _ = _frame_median(o1, c1, best["threads"])
    m1s, _ = _frame_median(o1, c1, 1)
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), None)
    except OSError:
        pass
    return {"value": best["value"], "unit": "Mrays/s", "cores": best["threads"], "kind": "port",
            "build": blib.oracle_build_info().decode(),
            "sample": f"{spec.name} {spec.width}x{spec.height} full frames ({rays} rays each): oracle/libbaseline.so "
                      f"per-ray traversal, {best['threads']} threads, 1 warm-up + median of 5 frames",
            "runs": runs, "single_thread": round(rays / med1 / 1e6, 3),
            "checker": {"value": round(rays / chk / 1e6, 3), "threads": best["threads"],
                        "build": "oracle/liboracle.so (-O2, counters on: the parity checker)"},
            "host_cpus": ncpu, "os_cpu_count": os.cpu_count(), "cgroup_cpu_quota": quota, "cpu_model": model,
            "wall_s": round(time.perf_counter() - t_all, 1),
            "C1": {"value": round(r1 / m1 / 1e6, 3), "unit": "Mrays/s", "cores": best["threads"],
                   "single_thread": round(r1 / m1s / 1e6, 3),
                   "sample": f"C1 512x512 primary only ({r1} rays), 1 warm-up + median of 5 frames"}}


def measure_raster(be, spec, steps: int, warmup: int) -> dict:
    """Raster fallback (rt_raster_draw: the reference's scrapped raster pipeline) on one GPU."""
    from realtimeraytracing_gradproject_amd import scenes
    W, H = spec.width, spec.height
    rt = be.rt
    with rt.Context(be.local) as ctx:
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
    return {"config": f"{spec.name} raster", "frame_ms": round(wall / steps * 1e3, 4), "gpu_ms": round(ms, 4),
            "triangles": int(tris), "resolution": f"{W}x{H}"}


def workload(spec) -> str:
    return (f"{spec.name}: {spec.model}.obj x{len(spec.instances) - 1} + plane, {len(spec.lights)} light(s), "
            f"{spec.width}x{spec.height}, {spec.spp} spp, shade {['ref', 'lambert_shadow', 'primary'][spec.mode]}")


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn(a, argv)
    if world > 1 and a.gpus != world:
        a.gpus = world
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    # --mode strips at N = 1: the tiled-frame loop over a world-1 communicator (rehearsal of the N > 1 path)
    strips = (distributed and a.mode in ("auto", "strips")) or a.mode == "strips"

    from realtimeraytracing_gradproject_amd import scenes
    be = make_backend(local)
    if distributed or strips:
        if not distributed:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        be.init_pg()

    def spec_of(name):
        s = scenes.config(name)
        if a.size:
            w, h = (int(v) for v in a.size.lower().split("x"))
            s = s.with_size(w, h)
        return s

    spec = spec_of(a.config)
    r = run_config(be, spec, world, rank, a.steps, a.warmup, a.settle_ms, strips, not a.no_pipeline, a.schedule,
                   a.save_image, a.in_flight, a.resettle_ms, a.frames_per_gather, a.frames_per_launch, a.loopback,
                   a.latency_frames, a.phase_frames)

    extra = []
    names = a.extra if a.extra is not None else ("C4,C5" if distributed else "C1,C2F,C3,C4,C5,REF")
    for name in [n for n in names.split(",") if n]:
        es = spec_of(name)
        # at least 50 frames (10 at 4 spp: C5 is ~4.4 ms per frame on one GPU): with the driver's 20 steps a quarter
        # of them was 5 frames, 70 us of C1, where the host's issue and synchronise dominated (C1 / C2F read 24-46 %
        # below their 200-step rates in BENCH_r03.json)
        n_steps = max(10, a.steps // 20) if es.spp > 1 else max(50, a.steps // 4)
        x = run_config(be, es, world, rank, n_steps, 2, 0.0, strips, not a.no_pipeline, a.schedule,
                       in_flight=a.in_flight, resettle_ms=a.resettle_ms, frames_per_gather=a.frames_per_gather,
                       frames_per_launch=a.frames_per_launch, loopback=a.loopback,
                       latency_frames=min(a.latency_frames, 5),
                       phase_frames=min(a.phase_frames, 16 if es.spp > 1 else 64))
        if rank == 0:
            st = x["stats"]
            rays = max(x["rays_step"], 1)
            extra.append({"config": name, "Mrays_s": round(x["rays_step"] * n_steps / x["tmax"] / 1e6, 1),
                          "frame_ms": round(x["tmax"] / n_steps * 1e3, 4), "kernel_ms": round(x["kernel_ms"], 4),
                          "rays_per_step": x["rays_step"], "resolution": f"{es.width}x{es.height}", "spp": es.spp,
                          "n_gpus": world, "parallelism": f"strips{world}+gather" if strips else f"frames{world}",
                          "tile_rows": x["tile_rows"], "frames_in_flight": x["in_flight"],
                          "frame_latency_ms": None if x["latency_ms"] is None else round(x["latency_ms"], 4),
                          "tile_balance": x["tile_balance"], "phases": x["phases"],
                          "aabb_tests_per_ray_rank0": round(st["aabb_tests"] / rays, 2) if not distributed else None,
                          "node_fetches": int(st["node_fetches"]), "tri_fetches": int(st["tri_fetches"])})
    if not distributed and (a.extra is None) and isinstance(be, HipBackend):
        extra.append(be.raster(scenes.config("REF"), max(5, a.steps // 4), 2))

    if rank == 0:
        W, H = spec.width, spec.height
        value = r["rays_step"] * a.steps / r["tmax"] / 1e6
        st = r["stats"]
        cpu = None
        if not distributed and not a.no_cpu_baseline:
            cpu = cpu_baseline(spec, a.cpu_seconds)
        rf = roofline(spec.name, st, W * r["rows_local"], r["kernel_ms"], a.schedule)
        if distributed:
            rf["note"] = "rank 0's strip render alone, timed back to back after the timed region"
        out = {
            "metric": "Mrays/sec (primary+shadow) at 1080p",
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(r["tmax"] / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if strips else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic camera/lights of BASELINE config; meshes teapot.obj/rabbit.obj from the reference",
            "config": {"workload": workload(spec), "rays_per_step": r["rays_step"],
                       "primary_rays": r["primary"], "shadow_rays": r["shadow"],
                       "parallelism": (f"strips{world}+gather" + ("" if a.no_pipeline else " (pipelined)")) if strips
                       else f"frames{world}",
                       "rccl_world_size": world if (distributed or strips) else None, "strips_loop": r["strips_loop"],
                       "frames_per_gather": r["fpg"], "frames_per_launch": r["fpl"],
                       "loopback_ranks": r["loopback"] or None,
                       # SURVEY 8(d)'s frame latency in strips mode: enqueue -> assembled on rank 0, gather included,
                       # one frame per gather, one at a time (the batched throughput is `value`)
                       "frame_latency_ms": None if r["latency_ms"] is None else round(r["latency_ms"], 4),
                       # what a step costs per phase on rank 0 (native strips loop; null otherwise)
                       "phases": r["phases"],
                       "schedule": a.schedule,
                       "tile_rows": r["tile_rows"], "tile_ms_rank0": r["tile_ms"],
                       "frames_in_flight": r["in_flight"], "in_flight_ms_rank0": r["in_flight_ms"],
                       # one frame alone on one stream, back to back (this rank's render; at N = 1 without strips
                       # this is SURVEY 8(d)'s frame latency: enqueue -> complete)
                       "frame_ms_one_stream": round(r["kernel_ms"], 4),
                       "frame_ms_one_stream_is_latency": not strips,
                       "tile_balance": r["tile_balance"],
                       "settle_ms": a.settle_ms, "resettle_ms": a.resettle_ms},
            "roofline": rf,
            "cpu_baseline": cpu,
            "build_ms": dict(zip(("blas", "tlas", "blas_warm", "tlas_warm", "tlas_update_wall", "tlas_update_kernel"),
                                 r["build"])),
            "extra": extra,
        }
        print(json.dumps(out), flush=True)
    be.close()
    if distributed or strips:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
