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
