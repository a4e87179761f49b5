"""Test-only bench backend (RT_BENCH_TEST_BACKEND=tests.bench_cpu_backend:CpuBackend): bench.py's
launcher, strip partition, gather, assembly, counter all-reduce and max-over-ranks timing run
unchanged on CPU tensors over gloo, with the CPU oracle as each rank's renderer (the only renderer
without a GPU). Never used by the product: bench.py's default backend is the HIP library."""
import contextlib
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import oracle  # noqa: E402  (checker)
import realtimeraytracing_gradproject_amd as rt  # noqa: E402
from realtimeraytracing_gradproject_amd import distributed as D  # noqa: E402


class _Stream:
    cuda_stream = None

    def wait_event(self, e):
        pass


class _WallEvent:
    def __init__(self):
        self.t = None

    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


class CpuBackend:
    dist_backend = "gloo"

    def __init__(self, local: int):
        self.local = local
        self.device = torch.device("cpu")
        self.renders = 0

    def init_pg(self):
        dist.init_process_group("gloo")

    def load(self, spec, schedule):
        self.spec = spec
        self.o = oracle.Scene(spec)
        self.schedule = 1 if schedule == "lane" else 0
        return [0.0] * len(spec.meshes), 0.0

    def zeros(self, shape):
        return torch.zeros(shape, dtype=torch.uint8)

    def stream(self):
        return _Stream()

    def event(self, timing=False):
        return _WallEvent()

    def use_stream(self, s):
        return contextlib.nullcontext()

    def sync_event(self):
        return _WallEvent()

    def record(self, ev, stream):
        ev.record(stream)

    def wait(self, stream, ev):
        pass

    def synchronize(self):
        pass

    def _render(self, buf, rows):
        o8, _, st = self.o.render_spec(self.spec, rows=rows, nthreads=2, want_float=False, schedule=self.schedule)
        buf[: o8.shape[0]] = torch.from_numpy(o8)
        self.renders += 1
        return st

    def dispatch(self, buf, rows, stream):
        self._render(buf, rows)

    def counted(self, buf, rows, stream):
        st = self._render(buf, rows)
        return {k: int(v) for k, v in zip(rt.STAT_NAMES, st)}

    def assemble(self, world, gathered, frame, stream):
        frame[:] = torch.from_numpy(D.assemble_host(gathered.numpy(), self.spec.height, world))

    def close(self):
        pass


class _CommAvailable:
    @staticmethod
    def comm_available():
        return True


class CpuBackendCommFails(CpuBackend):
    """The native strips loop requested and RCCL reported available, but rt_comm_init fails on rank 1 only
    (RCCL_FAIL_RANK): every rank must fall back to the torch.distributed strips loop together."""
    native_strips = True
    rt = _CommAvailable()

    def comm_open(self, world, rank):
        if rank == int(os.environ.get("RCCL_FAIL_RANK", "1")):
            raise RuntimeError("rt_comm_init: simulated RCCL failure")

        class _Comm:
            depth = 3

            def close(self):
                pass

            def abort(self):  # bench.py must abort (no draining collective) the communicator the other rank lacks
                print(f"comm aborted on rank {rank}", file=sys.stderr, flush=True)
        return _Comm()


class CpuBackendStepFails(CpuBackend):
    """The native strips loop at world 1 whose render call raises on its STEP_FAIL_AT-th call (an error mid-loop,
    with a partly filled batch pending): bench.py must abort the communicator (rt_comm_abort, no draining gather) and
    let the error propagate."""
    native_strips = True
    rt = _CommAvailable()

    def comm_open(self, world, rank):
        class _Comm:
            depth, batch = 3, 1

            def set_batch(self, b):
                self.batch = b

            def synchronize(self):
                pass

            def close(self):
                print("comm closed", file=sys.stderr, flush=True)

            def abort(self):
                print("comm aborted", file=sys.stderr, flush=True)
        self._calls = 0
        return _Comm()

    def render_strips(self, comm, frames, stream):
        self._calls += 1
        if self._calls == int(os.environ.get("STEP_FAIL_AT", "3")):
            raise RuntimeError("simulated render failure")


class CpuBackendNative(CpuBackend):
    """bench.py's native strips loop (rt_render_strips_frames) at world N over gloo: a stand-in communicator renders
    this rank's strips with the oracle, gathers them to rank 0 (torch.distributed gather) and assembles the frames
    there, timing each phase on the wall clock the way the library's phase timing reports them (rt_comm_phase_stats'
    fields). Exercises bench.py's phase pass and its max / min render share over the ranks."""
    native_strips = True
    rt = _CommAvailable()

    def comm_open(self, world, rank):
        be = self
        H = self.spec.height
        rows, padded = D.rank_rows(H, world, rank), D.padded_rows(H, world)

        class _Comm:
            depth, batch = 3, 1

            def __init__(self):
                self.on = False
                self.ps = {}

            def set_batch(self, b):
                self.batch = b

            def synchronize(self):
                pass

            def close(self):
                pass

            def abort(self):
                pass

            def set_phase_timing(self, on):
                self.on = bool(on)
                self.ps = dict.fromkeys(("frames", "renders", "render_ms", "gathers", "gather_ms", "assemblies",
                                         "assembly_ms", "host_us", "calls", "issue_us", "bytes_in", "bytes"), 0.0)

            def phase_stats(self):
                return dict(self.ps)

            def step(self, frames, n):
                t0 = time.perf_counter()
                local = torch.zeros((padded, be.spec.width, 4), dtype=torch.uint8)
                be._render(local, rows)
                t1 = time.perf_counter()
                bufs = [torch.zeros_like(local) for _ in range(world)] if rank == 0 else None
                dist.gather(local, bufs, dst=0)
                t2 = time.perf_counter()
                if rank == 0:
                    g = torch.stack(bufs)
                    for f in frames:
                        f[:] = torch.from_numpy(D.assemble_host(g.numpy(), H, world))
                t3 = time.perf_counter()
                if self.on:
                    for k, v in (("frames", n), ("renders", 1), ("render_ms", (t1 - t0) * 1e3), ("gathers", 1),
                                 ("gather_ms", (t2 - t1) * 1e3), ("assemblies", 1 if rank == 0 else 0),
                                 ("assembly_ms", (t3 - t2) * 1e3), ("host_us", (t3 - t0) * 1e6), ("calls", 1),
                                 ("bytes_in", local.numel() * (world - 1) if rank == 0 else 0),
                                 ("bytes", local.numel() * world)):
                        self.ps[k] += v
        return _Comm()

    def render_strips(self, comm, frames, stream):
        comm.step([f for f in frames if f is not None], len(frames))
