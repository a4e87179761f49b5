"""MI355X-native ray tracer — Python view of the C-ABI in include/rt_api.h.

The product is the HIP library ``lib/librtamd.so`` (gfx950 kernels + host C++). This module only
binds its C entry points with ctypes for tests and the bench; it never computes a frame itself and
there is no CPU fallback: if the library is missing, importing the package raises.

torch is imported first on purpose: it loads the HIP runtime that the library then shares, so
device pointers and hipStream_t handles from torch tensors are valid in the library.
"""
from __future__ import annotations

import ctypes
import gzip
import os
from typing import Iterable, Optional, Sequence

import numpy as np

try:  # share torch's HIP runtime when torch is present
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is part of the image
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
# RT_LIBRARY (diagnostics: tools/asan_check.sh's sanitizer build of the same library) overrides the path
LIB_PATH = os.environ.get("RT_LIBRARY") or os.path.join(_HERE, "lib", "librtamd.so")
ASSETS = os.path.join(_HERE, "assets")

RT_OK, RT_E_INVALID, RT_E_OOM, RT_E_HIP, RT_E_RCCL, RT_E_UNSUPPORTED, RT_E_IO = 0, -1, -2, -3, -4, -5, -6
RT_HITGROUP_MODEL, RT_HITGROUP_SHADOW, RT_HITGROUP_PLANE = 0, 1, 2
RT_SHADE_REF, RT_SHADE_LAMBERT_SHADOW, RT_SHADE_PRIMARY = 0, 1, 2
RT_SCHED_PACKET, RT_SCHED_LANE = 0, 1
RT_BALANCE_INFO_COUNT = 20
RT_RAY_FLAG_ACCEPT_FIRST_HIT_AND_END_SEARCH, RT_RAY_FLAG_CULL_BACK_FACING_TRIANGLES = 0x04, 0x10
RT_RAY_FLAG_CULL_FRONT_FACING_TRIANGLES = 0x20
STAT_NAMES = ("primary_rays", "shadow_rays", "aabb_tests", "tri_tests", "instance_entries",
              "stack_overflows", "pixels", "dispatches", "reflection_rays", "node_fetches", "tri_fetches",
              "instance_fetches")


class RtError(RuntimeError):
    """Non-zero rt_status (the reference's ThrowIfFailed, DXSampleHelper.h:16-22)."""

    def __init__(self, status: int, msg: str = ""):
        self.status = status
        super().__init__(f"{_status_name(status)}: {msg}" if msg else _status_name(status))


class rt_instance(ctypes.Structure):
    _fields_ = [("blas", ctypes.c_uint32), ("xform3x4_rowmajor", ctypes.c_float * 12),
                ("instance_id", ctypes.c_uint32), ("hit_group", ctypes.c_uint32)]


class rt_light(ctypes.Structure):
    _fields_ = [("color", ctypes.c_float * 3), ("position", ctypes.c_float * 3),
                ("intensity", ctypes.c_float)]


class rt_material(ctypes.Structure):
    _fields_ = [("albedo", ctypes.c_float * 3), ("roughness", ctypes.c_float),
                ("metallic", ctypes.c_float), ("reflectivity", ctypes.c_float)]


class rt_bvh_info(ctypes.Structure):
    _fields_ = [("prim_count", ctypes.c_uint32), ("node_count", ctypes.c_uint32),
                ("depth", ctypes.c_uint32), ("max_stack", ctypes.c_uint32),
                ("bounds_lo", ctypes.c_float * 3), ("bounds_hi", ctypes.c_float * 3),
                ("build_ms", ctypes.c_double)]


class rt_manipulator(ctypes.Structure):
    """include/rt_api.h rt_manipulator: nv_helpers_dx12::Manipulator state (manipulator.h:124-144)."""
    _fields_ = [("pos", ctypes.c_float * 3), ("interest", ctypes.c_float * 3), ("up", ctypes.c_float * 3),
                ("roll", ctypes.c_float), ("matrix", ctypes.c_float * 16), ("width", ctypes.c_int32),
                ("height", ctypes.c_int32), ("speed", ctypes.c_float), ("mouse", ctypes.c_float * 2),
                ("tbsize", ctypes.c_float), ("mode", ctypes.c_int32)]


_P = ctypes.c_void_p
_U32 = ctypes.c_uint32
_I = ctypes.c_int
_FP = ctypes.POINTER(ctypes.c_float)
_UP = ctypes.POINTER(ctypes.c_uint32)

# (name, restype, argtypes) — every function declared in include/rt_api.h
SIGNATURES = [
    ("rt_api_version", _I, []),
    ("rt_status_string", ctypes.c_char_p, [_I]),
    ("rt_last_error", ctypes.c_char_p, [_P]),
    ("rt_create", _I, [_I, ctypes.POINTER(_P)]),
    ("rt_destroy", _I, [_P]),
    ("rt_blas_build", _I, [_P, _P, _U32, _U32, _P, _U32, _UP]),
    ("rt_blas_rebuild", _I, [_P, _U32, _P, _U32, _U32, _P, _U32]),
    ("rt_blas_info", _I, [_P, _U32, ctypes.POINTER(rt_bvh_info)]),
    ("rt_blas_export", _I, [_P, _U32, _P, ctypes.c_size_t, _P, ctypes.c_size_t]),
    ("rt_tlas_build", _I, [_P, ctypes.POINTER(rt_instance), _U32, _I]),
    ("rt_tlas_info", _I, [_P, ctypes.POINTER(rt_bvh_info)]),
    ("rt_tlas_build_wall_ms", ctypes.c_double, [_P]),
    ("rt_tlas_export", _I, [_P, _P, ctypes.c_size_t]),
    ("rt_set_camera", _I, [_P, _FP]),
    ("rt_set_shading", _I, [_P, ctypes.POINTER(rt_light), _U32, ctypes.POINTER(rt_material), _I, _I]),
    ("rt_set_schedule", _I, [_P, _I]),
    ("rt_set_tile_rows", _I, [_P, _I]),
    ("rt_set_tile_balance", _I, [_P, _I]),
    ("rt_tile_balance_info", _I, [_P, _UP]),
    ("rt_tile_balance_info_n", _I, [_P, _UP, _U32]),
    ("rt_ctx_counters", _I, [_P, ctypes.POINTER(ctypes.c_uint64)]),
    ("rt_ctx_counters_n", _I, [_P, ctypes.POINTER(ctypes.c_uint64), _U32]),
    ("rt_set_stats", _I, [_P, _I]),
    ("rt_dispatch_rays", _I, [_P, _U32, _U32, _P, _U32, _P, _P, _P]),
    ("rt_dispatch_frames", _I, [_P, _U32, _U32, _U32, _P, _P, ctypes.c_uint64, _P]),
    ("rt_trace_rays", _I, [_P, _P, _U32, _U32, _P, _P, _P]),
    ("rt_raster_draw", _I, [_P, _UP, _U32, _FP, _U32, _U32, _P, _P, _P]),
    ("rt_assemble_strips", _I, [_P, _U32, _U32, _U32, _U32, _P, _P, _P]),
    ("rt_strip_rows", _U32, [_U32, _U32, _U32, _U32, _P, _U32]),
    ("rt_forget_stream", _I, [_P, _P]),
    ("rt_event_create", _I, [ctypes.POINTER(_P)]),
    ("rt_event_destroy", _I, [_P]),
    ("rt_event_record", _I, [_P, _P]),
    ("rt_stream_wait_event", _I, [_P, _P]),
    ("rt_comm_available", _I, []),
    ("rt_comm_get_unique_id", _I, [_P]),
    ("rt_comm_init", _I, [_P, _U32, _U32, _P, ctypes.POINTER(_P)]),
    ("rt_comm_init_loopback", _I, [_P, _U32, ctypes.POINTER(_P)]),
    ("rt_comm_destroy", _I, [_P]),
    ("rt_comm_abort", _I, [_P]),
    ("rt_comm_loopback_render_ranks", _I, [_P, _U32, _U32]),
    ("rt_comm_set_phase_timing", _I, [_P, ctypes.c_int]),
    ("rt_comm_phase_stats", _I, [_P, ctypes.POINTER(ctypes.c_double), _U32]),
    ("rt_comm_last_error", ctypes.c_char_p, [_P]),
    ("rt_comm_stream", _P, [_P]),
    ("rt_comm_synchronize", _I, [_P]),
    ("rt_render_strips", _I, [_P, _U32, _U32, _U32, _P, _P]),
    ("rt_render_strips_frames", _I, [_P, _U32, _U32, _U32, _U32, _FP, ctypes.POINTER(_P), _P]),
    ("rt_comm_pipeline_depth", _U32, [_P]),
    ("rt_comm_set_batch", _I, [_P, _U32]),
    ("rt_comm_batch", _U32, [_P]),
    ("rt_stats", _I, [_P, ctypes.POINTER(ctypes.c_uint64)]),
    ("rt_stats_reset", _I, [_P]),
    ("rt_mesh_load_obj", _I, [ctypes.c_char_p, ctypes.POINTER(_P)]),
    ("rt_mesh_parse_obj", _I, [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(_P)]),
    ("rt_mesh_free", None, [_P]),
    ("rt_mesh_vertex_count", _U32, [_P]),
    ("rt_mesh_index_count", _U32, [_P]),
    ("rt_mesh_vertices", _FP, [_P]),
    ("rt_mesh_indices", _UP, [_P]),
    ("rt_mesh_compute_vertex_normals", _I, [_P]),
    ("rt_plane_vertices", None, [_FP]),
    ("rt_camera_lookat", None, [_FP, _FP, _FP, _FP]),
    ("rt_camera_buffer", None, [_FP, _U32, _U32, ctypes.c_float, ctypes.c_float, ctypes.c_float, _FP]),
    ("rt_manip_init", None, [ctypes.POINTER(rt_manipulator)]),
    ("rt_manip_update", None, [ctypes.POINTER(rt_manipulator)]),
    ("rt_manip_set_lookat", None, [ctypes.POINTER(rt_manipulator), _FP, _FP, _FP]),
    ("rt_manip_set_roll", None, [ctypes.POINTER(rt_manipulator), ctypes.c_float]),
    ("rt_manip_set_window_size", None, [ctypes.POINTER(rt_manipulator), ctypes.c_int32, ctypes.c_int32]),
    ("rt_manip_set_mouse_position", None, [ctypes.POINTER(rt_manipulator), ctypes.c_int32, ctypes.c_int32]),
    ("rt_manip_motion", None, [ctypes.POINTER(rt_manipulator), ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    ("rt_manip_mouse_move", ctypes.c_int32, [ctypes.POINTER(rt_manipulator), ctypes.c_int32, ctypes.c_int32,
                                             ctypes.c_uint32]),
    ("rt_manip_wheel", None, [ctypes.POINTER(rt_manipulator), ctypes.c_int32]),
]


def _load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Loads the C-ABI library (a variant build may be given for A/B timing in one process)."""
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build the HIP library first "
            "(python -c 'import __graft_entry__ as g; g.build()' or `make`). There is no CPU fallback.")
    lib = ctypes.CDLL(path)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def _status_name(st: int) -> str:
    return lib.rt_status_string(st).decode()


def _fptr(a: np.ndarray):
    return a.ctypes.data_as(_FP)


def _f32(x, n=None) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float32))
    if n is not None and a.size != n:
        raise ValueError(f"expected {n} floats, got {a.size}")
    return a


# ---------------------------------------------------------------------------------------------
# host services (no GPU)
# ---------------------------------------------------------------------------------------------

class Mesh:
    """OBJFileManager::LoadObjFile result (OBJ_FileManager.cpp:10-71) held by the C library."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def load_obj(cls, path: str) -> "Mesh":
        h = _P()
        st = lib.rt_mesh_load_obj(path.encode(), ctypes.byref(h))
        if st != RT_OK:
            raise RtError(st, f"cannot load {path}")
        return cls(h)

    @classmethod
    def parse_obj(cls, text: bytes) -> "Mesh":
        h = _P()
        st = lib.rt_mesh_parse_obj(text, len(text), ctypes.byref(h))
        if st != RT_OK:
            raise RtError(st, "parse failed")
        return cls(h)

    @classmethod
    def asset(cls, name: str) -> "Mesh":
        """A model shipped with the package (teapot, rabbit), stored gzip-compressed."""
        with gzip.open(os.path.join(ASSETS, f"{name}.obj.gz"), "rb") as f:
            return cls.parse_obj(f.read())

    def __del__(self):
        if getattr(self, "_h", None) and lib is not None:
            lib.rt_mesh_free(self._h)
            self._h = None

    @property
    def vertex_count(self) -> int:
        return lib.rt_mesh_vertex_count(self._h)

    @property
    def index_count(self) -> int:
        return lib.rt_mesh_index_count(self._h)

    @property
    def vertices(self) -> np.ndarray:
        n = self.vertex_count
        if n == 0:
            return np.zeros((0, 6), np.float32)
        return np.ctypeslib.as_array(lib.rt_mesh_vertices(self._h), shape=(n * 6,)).reshape(n, 6).copy()

    @property
    def indices(self) -> np.ndarray:
        n = self.index_count
        if n == 0:
            return np.zeros((0,), np.uint32)
        return np.ctypeslib.as_array(lib.rt_mesh_indices(self._h), shape=(n,)).copy()

    def compute_vertex_normals(self) -> "Mesh":
        st = lib.rt_mesh_compute_vertex_normals(self._h)
        if st != RT_OK:
            raise RtError(st, "ComputeVertexNormals")
        return self


def plane_vertices() -> np.ndarray:
    out = np.zeros(36, np.float32)
    lib.rt_plane_vertices(_fptr(out))
    return out.reshape(6, 6)


def camera_lookat(eye, center, up) -> np.ndarray:
    e, c, u = _f32(eye, 3), _f32(center, 3), _f32(up, 3)
    out = np.zeros(16, np.float32)
    lib.rt_camera_lookat(_fptr(e), _fptr(c), _fptr(u), _fptr(out))
    return out


def camera_buffer(view, width: int, height: int, fov_deg: float = 45.0, znear: float = 0.1,
                  zfar: float = 1000.0) -> np.ndarray:
    v = _f32(view, 16)
    out = np.zeros(64, np.float32)
    lib.rt_camera_buffer(_fptr(v), width, height, fov_deg, znear, zfar, _fptr(out))
    return out


class Manipulator:
    """Camera manipulator with the reference's API (nv_helpers_dx12::Manipulator,
    include/manipulator.h:33-148, src/manipulator.cpp) over the C-ABI rt_manip_* functions.
    Host-only arithmetic; results are bit-identical to the reference's glm arithmetic."""
    Examine, Fly, Walk, Trackball = 0, 1, 2, 3          # Modes, manipulator.h:37
    NoAction, Orbit, Dolly, Pan, LookAround = 0, 1, 2, 3, 4  # Actions, manipulator.h:38
    LMB, MMB, RMB, SHIFT, CTRL, ALT = 0x01, 0x02, 0x04, 0x08, 0x10, 0x20  # Inputs bits

    def __init__(self):
        self._m = rt_manipulator()
        lib.rt_manip_init(ctypes.byref(self._m))

    @staticmethod
    def inputs(lmb=False, mmb=False, rmb=False, shift=False, ctrl=False, alt=False) -> int:
        """Manipulator::Inputs (manipulator.h:39-40) -> RT_INPUT_* bits."""
        return (lmb * 0x01) | (mmb * 0x02) | (rmb * 0x04) | (shift * 0x08) | (ctrl * 0x10) | (alt * 0x20)

    def setLookat(self, eye, center, up):
        e, c, u = _f32(eye, 3), _f32(center, 3), _f32(up, 3)
        lib.rt_manip_set_lookat(ctypes.byref(self._m), _fptr(e), _fptr(c), _fptr(u))

    def getLookat(self):
        m = self._m
        return (np.array(m.pos[:], np.float32), np.array(m.interest[:], np.float32), np.array(m.up[:], np.float32))

    def setWindowSize(self, w: int, h: int):
        lib.rt_manip_set_window_size(ctypes.byref(self._m), w, h)

    def getWidth(self) -> int:
        return self._m.width

    def getHeight(self) -> int:
        return self._m.height

    def setMousePosition(self, x: int, y: int):
        lib.rt_manip_set_mouse_position(ctypes.byref(self._m), x, y)

    def getMousePosition(self):
        return int(self._m.mouse[0]), int(self._m.mouse[1])

    def setMode(self, mode: int):
        self._m.mode = mode

    def getMode(self) -> int:
        return self._m.mode

    def setRoll(self, roll: float):
        lib.rt_manip_set_roll(ctypes.byref(self._m), roll)

    def getRoll(self) -> float:
        return self._m.roll

    def setSpeed(self, speed: float):
        self._m.speed = speed

    def getSpeed(self) -> float:
        return self._m.speed

    def getMatrix(self) -> np.ndarray:
        """Column-major 4x4 as glm stores it (16 floats)."""
        return np.array(self._m.matrix[:], np.float32)

    def motion(self, x: int, y: int, action: int = 0):
        lib.rt_manip_motion(ctypes.byref(self._m), x, y, action)

    def mouseMove(self, x: int, y: int, inputs: int) -> int:
        return int(lib.rt_manip_mouse_move(ctypes.byref(self._m), x, y, inputs))

    def wheel(self, value: int):
        lib.rt_manip_wheel(ctypes.byref(self._m), value)


def strip_rows(height: int, nranks: int, rank: int, strip_rows_: int = 8) -> np.ndarray:
    n = lib.rt_strip_rows(height, nranks, rank, strip_rows_, None, 0)
    out = np.zeros(n, np.uint32)
    lib.rt_strip_rows(height, nranks, rank, strip_rows_, out.ctypes.data_as(_P), n)
    return out


class PipelineEvent:
    """rt_event_*: a device-side sync point between the strips loop's render and gather streams
    (no timestamp, no system-scope fence on record). record(stream) / wait_on(stream) take raw
    hipStream_t handles (torch: stream.cuda_stream)."""

    def __init__(self):
        h = _P()
        st = lib.rt_event_create(ctypes.byref(h))
        if st != RT_OK:
            raise RtError(st, "rt_event_create")
        self._h = h

    def record(self, stream: Optional[int]):
        st = lib.rt_event_record(self._h, stream)
        if st != RT_OK:
            raise RtError(st, "rt_event_record")

    def wait_on(self, stream: Optional[int]):
        """Later work on `stream` waits for this event's last record."""
        st = lib.rt_stream_wait_event(stream, self._h)
        if st != RT_OK:
            raise RtError(st, "rt_stream_wait_event")

    def close(self):
        if self._h:
            lib.rt_event_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001  (interpreter shutdown)
            pass


RT_COMM_ID_BYTES = 128


def comm_available() -> bool:
    """rt_comm_available: RCCL can be loaded (no collective, no GPU work)."""
    return lib.rt_comm_available() == RT_OK


def comm_unique_id() -> bytes:
    """rt_comm_get_unique_id (ncclGetUniqueId): created on rank 0, handed to every rank by the caller."""
    buf = ctypes.create_string_buffer(RT_COMM_ID_BYTES)
    st = lib.rt_comm_get_unique_id(buf)
    if st != RT_OK:
        raise RtError(st, "rt_comm_get_unique_id")
    return buf.raw


class Comm:
    """rt_comm_*: the native multi-GPU frame loop (strips -> ncclGather -> assembly on rank 0) of one context.
    Collective: every rank constructs it with the same 128-byte id and calls render_strips in the same order."""

    def __init__(self, ctx: "Context", nranks: int, rank: int, uid: Optional[bytes]):
        """uid None: a loopback communicator (rt_comm_init_loopback, tests): this process renders every one of
        the nranks ranks on its one GPU and the gather is a device copy (rank must be 0)."""
        self._lib = ctx._lib
        self.ctx, self.nranks, self.rank = ctx, nranks, rank
        self.is_loopback = uid is None
        self._pending = False  # frames handed to render_strips* since the last synchronize (a partly filled batch)
        h = _P()
        if uid is None:
            if rank != 0:
                raise ValueError("a loopback communicator is rank 0")
            st = self._lib.rt_comm_init_loopback(ctx._h, nranks, ctypes.byref(h))
            if st != RT_OK:
                raise RtError(st, f"rt_comm_init_loopback(nranks={nranks})")
            self._h = h
            return
        if len(uid) != RT_COMM_ID_BYTES:
            raise ValueError("the communicator id is 128 bytes")
        self._idbuf = ctypes.create_string_buffer(uid, RT_COMM_ID_BYTES)
        st = self._lib.rt_comm_init(ctx._h, nranks, rank, self._idbuf, ctypes.byref(h))
        if st != RT_OK:
            raise RtError(st, f"rt_comm_init(nranks={nranks}, rank={rank})")
        self._h = h

    @classmethod
    def loopback(cls, ctx: "Context", nranks: int) -> "Comm":
        """rt_comm_init_loopback: nranks ranks emulated by this process on its one GPU (no RCCL)."""
        return cls(ctx, nranks, 0, None)

    def _check(self, st: int, what: str):
        if st != RT_OK:
            raise RtError(st, f"{what}: {self._lib.rt_comm_last_error(self._h).decode()}")

    def render_strips(self, width: int, height: int, frame_out=None, stream: Optional[int] = None,
                      strip_rows_: int = 8):
        """One tiled frame (rt_render_strips): frame_out is rank 0's H x W x 4 device buffer."""
        self._pending = True
        self._check(self._lib.rt_render_strips(self._h, width, height, strip_rows_, _ptr(frame_out), stream),
                    "rt_render_strips")

    def render_strips_frames(self, width: int, height: int, frames_out, cameras=None, stream: Optional[int] = None,
                             strip_rows_: int = 8):
        """rt_render_strips_frames: len(frames_out) frames in one launch per rank (cameras: n x 64 floats or None =
        the context's camera); frames_out: rank 0's device buffers (None entries on other ranks)."""
        n = len(frames_out)
        ptrs = (_P * n)(*[_ptr(f) for f in frames_out])
        cams = None if cameras is None else _f32(cameras, 64 * n)
        self._pending = True
        self._check(self._lib.rt_render_strips_frames(self._h, width, height, strip_rows_, n,
                                                      None if cams is None else _fptr(cams), ptrs, stream),
                    "rt_render_strips_frames")

    @property
    def stream(self) -> int:
        """hipStream_t of the gathers, made to wait for every step issued so far (rt_comm_stream)."""
        return self._lib.rt_comm_stream(self._h)

    @property
    def depth(self) -> int:
        """Frames in the pipeline: slots (one render stream each) x frames per gather; a caller that gives each
        call its own frame buffer needs this many to never wait on a frame buffer's previous assembly."""
        return int(self._lib.rt_comm_pipeline_depth(self._h))

    def set_batch(self, frames_per_gather: int):
        """rt_comm_set_batch: frames whose strips go in one ncclGather (every rank the same, between the same calls)."""
        self._check(self._lib.rt_comm_set_batch(self._h, frames_per_gather), "rt_comm_set_batch")

    @property
    def batch(self) -> int:
        return int(self._lib.rt_comm_batch(self._h))

    def synchronize(self):
        self._check(self._lib.rt_comm_synchronize(self._h), "rt_comm_synchronize")
        self._pending = False

    def close(self):
        """rt_comm_destroy: drains the pipeline (a partly filled batch included), then frees the communicator.
        Collective for an RCCL communicator: EVERY rank must call close() (or every rank abort()); a rank that drops
        its communicator unclosed aborts it (__del__), and a peer draining a partly filled batch would then wait for
        a gather that rank never issues."""
        if getattr(self, "_h", None):
            h, self._h = self._h, None
            st = self._lib.rt_comm_destroy(h)
            if st != RT_OK:
                raise RtError(st, "rt_comm_destroy")

    def set_phase_timing(self, on: bool):
        """rt_comm_set_phase_timing: timing-event pairs around each step's render, gather and assembly (drains)."""
        self._check(self._lib.rt_comm_set_phase_timing(self._h, 1 if on else 0), "rt_comm_set_phase_timing")
        self._pending = False

    def phase_stats(self) -> dict:
        """rt_comm_phase_stats: the phase sums since set_phase_timing(True) (drains the pipeline)."""
        out = (ctypes.c_double * 12)()
        self._check(self._lib.rt_comm_phase_stats(self._h, out, 12), "rt_comm_phase_stats")
        self._pending = False
        return dict(zip(("frames", "renders", "render_ms", "gathers", "gather_ms", "assemblies", "assembly_ms",
                         "host_us", "calls", "issue_us", "bytes_in", "bytes"), list(out)))

    def loopback_render_ranks(self, first: int = 0, count: int = 0):
        """rt_comm_loopback_render_ranks: a loopback communicator renders only emulated ranks [first, first + count)
        (0: all) — the rehearsal of one rank's share of a step; the other ranks' strips are stale."""
        self._check(self._lib.rt_comm_loopback_render_ranks(self._h, first, count), "rt_comm_loopback_render_ranks")

    def abort(self):
        """rt_comm_abort: the failure path. Frees the communicator without another collective (the partly filled
        batch is discarded, ncclCommAbort cancels gathers in flight): safe when other ranks may never call again."""
        if getattr(self, "_h", None):
            h, self._h = self._h, None
            st = self._lib.rt_comm_abort(h)
            if st != RT_OK:
                raise RtError(st, "rt_comm_abort")

    def __enter__(self):
        return self

    def __exit__(self, exc_type, exc, tb):
        # a normal exit drains (collective); an exception may have left the ranks out of step: abort
        if exc_type is None:
            self.close()
        else:
            self.abort()
        return False

    def __del__(self):
        # An unclosed communicator is garbage. Loopback: no peers, so it drains like close() (frames already handed
        # to render_strips are rendered and assembled). RCCL: the other ranks may not issue the collective a
        # draining destroy would need (an exception path, interpreter shutdown), so it aborts -- and says so when
        # that discards frames (close() is required on every rank).
        if not getattr(self, "_h", None):
            return
        try:
            if self.is_loopback:
                self.close()
                return
            if self._pending:
                import warnings
                warnings.warn("rt.Comm garbage-collected unclosed with frames pending: aborted (their partly filled "
                              "batch is discarded); call close() on every rank", ResourceWarning, stacklevel=2)
            self.abort()
        except Exception:  # noqa: BLE001  (interpreter shutdown)
            pass


def strip_rows_per_rank(height: int, nranks: int, strip_rows_: int = 8) -> int:
    """Rows of the padded per-rank buffer that rt_assemble_strips expects (rank-major blocks)."""
    nstrips = (height + strip_rows_ - 1) // strip_rows_
    return ((nstrips + nranks - 1) // nranks) * strip_rows_


# ---------------------------------------------------------------------------------------------
# device context
# ---------------------------------------------------------------------------------------------

def _ptr(x) -> Optional[int]:
    """Device pointer of a torch tensor, an int address, or None."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    return x.data_ptr()


class Context:
    """One rt_ctx (one HIP device, one host thread)."""

    def __init__(self, device: int = 0, library: Optional[ctypes.CDLL] = None):
        self._lib = library if library is not None else lib
        h = _P()
        st = self._lib.rt_create(device, ctypes.byref(h))
        if st != RT_OK:
            raise RtError(st, f"rt_create(device={device})")
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None) and getattr(self, "_lib", None) is not None:
            self._lib.rt_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, st: int, what: str):
        if st != RT_OK:
            raise RtError(st, f"{what}: {self._lib.rt_last_error(self._h).decode()}")

    # acceleration structures ------------------------------------------------------------------
    def blas_build(self, vertices: np.ndarray, indices: Optional[np.ndarray] = None) -> int:
        v = np.ascontiguousarray(vertices, dtype=np.float32)
        stride = v.shape[1] * 4 if v.ndim == 2 else 24
        nv = v.shape[0] if v.ndim == 2 else v.size // 6
        out = _U32()
        if indices is None:
            st = self._lib.rt_blas_build(self._h, v.ctypes.data_as(_P), nv, stride, None, 0, ctypes.byref(out))
        else:
            i = np.ascontiguousarray(indices, dtype=np.uint32)
            st = self._lib.rt_blas_build(self._h, v.ctypes.data_as(_P), nv, stride, i.ctypes.data_as(_P), i.size,
                                   ctypes.byref(out))
        self._check(st, "rt_blas_build")
        return out.value

    def blas_rebuild(self, blas: int, vertices: np.ndarray, indices: Optional[np.ndarray] = None):
        v = np.ascontiguousarray(vertices, dtype=np.float32)
        stride = v.shape[1] * 4
        if indices is None:
            st = self._lib.rt_blas_rebuild(self._h, blas, v.ctypes.data_as(_P), v.shape[0], stride, None, 0)
        else:
            i = np.ascontiguousarray(indices, dtype=np.uint32)
            st = self._lib.rt_blas_rebuild(self._h, blas, v.ctypes.data_as(_P), v.shape[0], stride,
                                     i.ctypes.data_as(_P), i.size)
        self._check(st, "rt_blas_rebuild")

    def blas_info(self, blas: int) -> rt_bvh_info:
        info = rt_bvh_info()
        self._check(self._lib.rt_blas_info(self._h, blas, ctypes.byref(info)), "rt_blas_info")
        return info

    def blas_export(self, blas: int):
        info = self.blas_info(blas)
        nodes = np.zeros(info.node_count * 32, np.uint32)  # 128-B 4-wide nodes
        tris = np.zeros(info.prim_count * 12, np.uint32)
        self._check(self._lib.rt_blas_export(self._h, blas, nodes.ctypes.data_as(_P), nodes.nbytes,
                                             tris.ctypes.data_as(_P), tris.nbytes), "rt_blas_export")
        return nodes.reshape(-1, 32), tris.reshape(-1, 12)

    def tlas_build(self, instances: Sequence[tuple], update_only: bool = False):
        """instances: (blas, xform3x4 (12 floats), instance_id, hit_group) tuples."""
        arr = (rt_instance * len(instances))()
        for k, (b, x, iid, hg) in enumerate(instances):
            arr[k].blas = b
            arr[k].xform3x4_rowmajor[:] = [float(v) for v in np.asarray(x, np.float32).ravel()]
            arr[k].instance_id = iid
            arr[k].hit_group = hg
        self._check(self._lib.rt_tlas_build(self._h, arr, len(instances), 1 if update_only else 0), "rt_tlas_build")

    def tlas_info(self) -> rt_bvh_info:
        info = rt_bvh_info()
        self._check(self._lib.rt_tlas_info(self._h, ctypes.byref(info)), "rt_tlas_info")
        return info

    def tlas_build_wall_ms(self) -> float:
        """Host wall time of the last tlas_build (ms)."""
        return float(self._lib.rt_tlas_build_wall_ms(self._h))

    def tlas_export(self) -> np.ndarray:
        info = self.tlas_info()
        nodes = np.zeros(info.node_count * 32, np.uint32)
        self._check(self._lib.rt_tlas_export(self._h, nodes.ctypes.data_as(_P), nodes.nbytes), "rt_tlas_export")
        return nodes.reshape(-1, 32)

    # frame state ------------------------------------------------------------------------------
    def set_camera(self, cb: np.ndarray):
        c = _f32(cb, 64)
        self._check(self._lib.rt_set_camera(self._h, _fptr(c)), "rt_set_camera")

    def set_shading(self, lights: Iterable, material, mode: int, spp: int = 1):
        lights = list(lights)
        arr = (rt_light * len(lights))()
        for k, (col, pos, inten) in enumerate(lights):
            arr[k].color[:] = [float(v) for v in col]
            arr[k].position[:] = [float(v) for v in pos]
            arr[k].intensity = float(inten)
        m = rt_material()
        m.albedo[:] = [float(v) for v in material[0:3]]
        m.roughness, m.metallic, m.reflectivity = (float(v) for v in material[3:6])
        self._check(self._lib.rt_set_shading(self._h, arr, len(lights), ctypes.byref(m), mode, spp), "rt_set_shading")

    def set_schedule(self, schedule: int):
        self._check(self._lib.rt_set_schedule(self._h, schedule), "rt_set_schedule")

    def set_tile_rows(self, rows: int):
        """rt_set_tile_rows: 8 (8 x 8 pixel tiles per wave, default) or 4 (8 x 4)."""
        self._check(self._lib.rt_set_tile_rows(self._h, rows), "rt_set_tile_rows")

    def set_tile_balance(self, mode: int):
        """rt_set_tile_balance: 0 off, 1 adaptive (default), 2 / 3 / 4 / 5 forced split layouts (tests)."""
        self._check(self._lib.rt_set_tile_balance(self._h, mode), "rt_set_tile_balance")

    def tile_balance_info(self) -> dict:
        out = (ctypes.c_uint32 * RT_BALANCE_INFO_COUNT)()
        self._check(self._lib.rt_tile_balance_info_n(self._h, out, RT_BALANCE_INFO_COUNT), "rt_tile_balance_info_n")
        return dict(zip(("plans", "split", "items", "extra_cap", "max_ticks", "mean_ticks", "threshold", "launches",
                         "pays", "check_bad", "check_first_tile", "check_first_word", "plan_load_ticks",
                         "plan_budget_ticks", "plan_place_ticks", "slots", "refused", "refused_plans"), list(out)))

    def counters(self) -> dict:
        """rt_ctx_counters_n: device-wide synchronisations, tile-balance maps recycled / full, maps held, recycled maps
        that reached a plan."""
        out = (ctypes.c_uint64 * 5)()
        self._check(self._lib.rt_ctx_counters_n(self._h, out, 5), "rt_ctx_counters_n")
        return dict(zip(("device_syncs", "balance_recycled", "balance_full", "balance_maps", "balance_recycled_planned"),
                        list(out)))

    def set_stats(self, on: bool):
        self._check(self._lib.rt_set_stats(self._h, 1 if on else 0), "rt_set_stats")

    def stats(self) -> dict:
        out = (ctypes.c_uint64 * len(STAT_NAMES))()
        self._check(self._lib.rt_stats(self._h, out), "rt_stats")
        return dict(zip(STAT_NAMES, list(out)))

    def stats_reset(self):
        self._check(self._lib.rt_stats_reset(self._h), "rt_stats_reset")

    # launches ---------------------------------------------------------------------------------
    def dispatch(self, width: int, height: int, rgba8, rgba32f=None, rows: Optional[np.ndarray] = None,
                 stream: Optional[int] = None):
        if rows is not None:
            r = np.ascontiguousarray(rows, dtype=np.uint32)
            rp, nr = r.ctypes.data_as(_P), r.size
        else:
            rp, nr = None, height
        self._check(self._lib.rt_dispatch_rays(self._h, width, height, rp, nr, _ptr(rgba8), _ptr(rgba32f), stream),
                    "rt_dispatch_rays")

    def dispatch_frames(self, width: int, height: int, rgba8, cameras=None, stream: Optional[int] = None,
                        frame_stride: int = 0):
        """rt_dispatch_frames: len(rgba8) (1..4) full frames in one launch. rgba8: an (n, H, W, 4) uint8 device
        tensor (frames back to back, or frame_stride bytes apart); cameras: n x 64 floats (None: the context's
        camera for every frame)."""
        n = int(rgba8.shape[0])
        cams = None if cameras is None else _f32(cameras, 64 * n)
        self._pending = True
        self._check(self._lib.rt_dispatch_frames(self._h, width, height, n, None if cams is None else _fptr(cams),
                                                 _ptr(rgba8), frame_stride, stream), "rt_dispatch_frames")

    def trace_rays(self, rays, n: int, any_hit: bool, hits, uv=None, stream: Optional[int] = None,
                   cull_back: bool = False, cull_front: bool = False):
        flags = (RT_RAY_FLAG_ACCEPT_FIRST_HIT_AND_END_SEARCH if any_hit else 0) | \
            (RT_RAY_FLAG_CULL_BACK_FACING_TRIANGLES if cull_back else 0) | \
            (RT_RAY_FLAG_CULL_FRONT_FACING_TRIANGLES if cull_front else 0)
        self._check(self._lib.rt_trace_rays(self._h, _ptr(rays), n, flags, _ptr(hits), _ptr(uv), stream),
                    "rt_trace_rays")

    def raster_draw(self, draws: Sequence[int], width: int, height: int, rgba8, depth=None, object_to_world=None,
                    stream: Optional[int] = None):
        """Raster fallback (rt_raster_draw; shaders/shaders.hlsl:41-59, D3D12HelloTriangle.cpp:513-540):
        draws the BLAS vertex buffers in order with the current camera into rgba8 (H x W x 4 device
        tensor) and optionally depth (H x W float32 device tensor)."""
        d = np.ascontiguousarray(draws, dtype=np.uint32)
        x = None if object_to_world is None else _f32(object_to_world, 12)
        self._check(self._lib.rt_raster_draw(self._h, d.ctypes.data_as(_UP), len(d),
                                             None if x is None else _fptr(x), width, height, _ptr(rgba8),
                                             _ptr(depth), stream), "rt_raster_draw")

    def forget_stream(self, stream: int):
        """rt_forget_stream: call before destroying a stream this context launched on (see rt_api.h)."""
        self._check(self._lib.rt_forget_stream(self._h, stream), "rt_forget_stream")

    def assemble_strips(self, width: int, height: int, nranks: int, strip_rows_: int, gathered, out,
                        stream: Optional[int] = None):
        self._check(self._lib.rt_assemble_strips(self._h, width, height, nranks, strip_rows_, _ptr(gathered), _ptr(out),
                                           stream), "rt_assemble_strips")
