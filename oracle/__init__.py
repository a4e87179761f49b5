"""CPU ORACLE — test infrastructure only.

ctypes binding of oracle/liboracle.so (oracle/rt_oracle.c), the scalar C restatement of the
reference path. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker / the timed CPU baseline. The product never imports it.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# ORACLE_LIBRARY (tools/asan_check.sh: the checker built with the address / undefined-behaviour sanitizers)
LIB_PATH = os.environ.get("ORACLE_LIBRARY") or os.path.join(_HERE, "liboracle.so")

_P = ctypes.c_void_p
_U32 = ctypes.c_uint32
_I = ctypes.c_int
_FP = ctypes.POINTER(ctypes.c_float)


class oracle_instance(ctypes.Structure):
    _fields_ = [("blas", _U32), ("xform", ctypes.c_float * 12), ("instance_id", _U32), ("hit_group", _U32)]


class oracle_light(ctypes.Structure):
    _fields_ = [("color", ctypes.c_float * 3), ("position", ctypes.c_float * 3), ("intensity", ctypes.c_float)]


_SIGS = [
    ("oracle_obj_parse", _I, [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(_FP), ctypes.POINTER(_U32),
                              ctypes.POINTER(ctypes.POINTER(_U32)), ctypes.POINTER(_U32)]),
    ("oracle_free", None, [_P]),
    ("oracle_vertex_normals", _I, [_FP, _U32, _P, _U32]),
    ("oracle_camera_lookat", None, [_FP, _FP, _FP, _FP]),
    ("oracle_camera_buffer", None, [_FP, _U32, _U32, ctypes.c_float, ctypes.c_float, ctypes.c_float, _FP]),
    ("oracle_scene_create", _P, []),
    ("oracle_scene_destroy", None, [_P]),
    ("oracle_add_blas", _I, [_P, _FP, _U32, _P, _U32]),
    ("oracle_set_instances", _I, [_P, ctypes.POINTER(oracle_instance), _U32]),
    ("oracle_blas_info", _I, [_P, _I, _P]),
    ("oracle_tlas_info", _I, [_P, _P]),
    ("oracle_export_blas", _I, [_P, _I, _P, _P]),
    ("oracle_export_tlas", _I, [_P, _P]),
    ("oracle_render", _I, [_P, _FP, ctypes.POINTER(oracle_light), _U32, _FP, _I, _I, _U32, _U32, _P, _U32, _P, _P,
                           _I, _P, _I, _I]),
    ("oracle_render_split", _I, [_P, _FP, ctypes.POINTER(oracle_light), _U32, _FP, _I, _I, _U32, _U32, _P, _U32, _P,
                                 _P, _I, _P, _I, _I, _I]),
    ("oracle_trace_rays", _I, [_P, _P, _U32, _U32, _P, _P, _I, _P]),
    ("oracle_raster", _I, [_P, _P, _P, _P, _U32, _P, _P, _U32, _U32, _P, _P, _P]),
    ("oracle_pbr", None, [_FP, _FP, _FP, ctypes.POINTER(oracle_light), _U32, _FP, _FP]),
    ("oracle_direct", None, [_FP, _FP, ctypes.POINTER(oracle_light), _U32, _FP, _FP]),
    ("oracle_pow", ctypes.c_float, [ctypes.c_float, ctypes.c_float]),
    ("oracle_max_stack_reached", _I, [_I]),
    ("oracle_camera_rays", None, [_FP, _U32, _U32, _P, _P, _U32, ctypes.c_float, ctypes.c_float, _P]),
]


BASELINE_PATH = os.path.join(_HERE, "libbaseline.so")


def _load(path=LIB_PATH, sigs=None):
    if not os.path.exists(path):
        raise ImportError(f"{path} missing: run `make {os.path.relpath(path, os.path.dirname(_HERE))}`")
    lib = ctypes.CDLL(path)
    for n, r, a in (sigs if sigs is not None else _SIGS):
        f = getattr(lib, n)
        f.restype = r
        f.argtypes = a
    return lib


lib = _load()
_baseline = None


def baseline_lib():
    """oracle/libbaseline.so: the same C restatement built as BASELINE.md section 3's CPU baseline
    (-O3, counters compiled out; identical frames). Loaded on first use (bench.py's cpu_baseline leg)."""
    global _baseline
    if _baseline is None:
        _baseline = _load(BASELINE_PATH, _SIGS + [("oracle_build_info", ctypes.c_char_p, [])])
    return _baseline


def _f(a):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a, a.ctypes.data_as(_FP)


def obj_parse(text: bytes):
    v = _FP()
    nv = _U32()
    i = ctypes.POINTER(_U32)()
    ni = _U32()
    if lib.oracle_obj_parse(text, len(text), ctypes.byref(v), ctypes.byref(nv), ctypes.byref(i), ctypes.byref(ni)):
        raise RuntimeError("oracle_obj_parse failed")
    verts = np.ctypeslib.as_array(v, shape=(max(nv.value, 1) * 6,))[: nv.value * 6].reshape(-1, 6).copy()
    idx = np.ctypeslib.as_array(i, shape=(max(ni.value, 1),))[: ni.value].copy()
    lib.oracle_free(ctypes.cast(v, _P))
    lib.oracle_free(ctypes.cast(i, _P))
    return verts, idx


def vertex_normals(verts: np.ndarray, idx: np.ndarray) -> np.ndarray:
    v = np.ascontiguousarray(verts, dtype=np.float32).copy()
    i = np.ascontiguousarray(idx, dtype=np.uint32)
    if lib.oracle_vertex_normals(v.ctypes.data_as(_FP), v.shape[0], i.ctypes.data_as(_P), i.size):
        raise RuntimeError("oracle_vertex_normals failed")
    return v


def camera_lookat(eye, center, up) -> np.ndarray:
    out = np.zeros(16, np.float32)
    e, ep = _f(eye)
    c, cp = _f(center)
    u, up_ = _f(up)
    lib.oracle_camera_lookat(ep, cp, up_, out.ctypes.data_as(_FP))
    return out


def camera_buffer(view, W, H, fov=45.0, zn=0.1, zf=1000.0) -> np.ndarray:
    out = np.zeros(64, np.float32)
    v, vp = _f(view)
    lib.oracle_camera_buffer(vp, W, H, fov, zn, zf, out.ctypes.data_as(_FP))
    return out


def _lights(lights):
    arr = (oracle_light * len(lights))()
    for k, (c, p, it) in enumerate(lights):
        arr[k].color[:] = [float(x) for x in c]
        arr[k].position[:] = [float(x) for x in p]
        arr[k].intensity = float(it)
    return arr


def pbr(n, cam, P, lights, material):
    out = np.zeros(3, np.float32)
    a, ap = _f(n)
    b, bp = _f(cam)
    c, cp = _f(P)
    m, mp = _f(material)
    lib.oracle_pbr(ap, bp, cp, _lights(lights), len(lights), mp, out.ctypes.data_as(_FP))
    return out


def direct(n, P, lights, albedo):
    out = np.zeros(3, np.float32)
    a, ap = _f(n)
    c, cp = _f(P)
    m, mp = _f(albedo)
    lib.oracle_direct(ap, cp, _lights(lights), len(lights), mp, out.ctypes.data_as(_FP))
    return out


def raster(draws, cb, W: int, H: int, object_to_world=None):
    """Raster fallback oracle (rt_raster_oracle.c). draws: sequence of (vtx6 (n, 6) float32, idx or
    None) in submission order. Returns (rgba8 (H, W, 4), depth (H, W), prim (H, W) uint32)."""
    vs = [np.ascontiguousarray(v, dtype=np.float32).reshape(-1, 6) for v, _ in draws]
    ids = [None if i is None else np.ascontiguousarray(i, dtype=np.uint32).ravel() for _, i in draws]
    n = len(draws)
    vp = (ctypes.c_void_p * n)(*[v.ctypes.data for v in vs])
    ip = (ctypes.c_void_p * n)(*[None if i is None else i.ctypes.data for i in ids])
    nv = np.array([v.shape[0] for v in vs], np.uint32)
    nt = np.array([(v.shape[0] if i is None else i.size) // 3 for v, i in zip(vs, ids)], np.uint32)
    x = np.asarray([1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0] if object_to_world is None else object_to_world,
                   np.float32).ravel()
    c = np.ascontiguousarray(cb, dtype=np.float32).ravel()
    rgba8 = np.zeros((H, W, 4), np.uint8)
    depth = np.zeros((H, W), np.float32)
    prim = np.zeros((H, W), np.uint32)
    r = lib.oracle_raster(ctypes.cast(vp, _P), nv.ctypes.data_as(_P), ctypes.cast(ip, _P), nt.ctypes.data_as(_P), n,
                          x.ctypes.data_as(_P), c.ctypes.data_as(_P), W, H, rgba8.ctypes.data_as(_P),
                          depth.ctypes.data_as(_P), prim.ctypes.data_as(_P))
    if r:
        raise RuntimeError(f"oracle_raster failed ({r})")
    return rgba8, depth, prim


def camera_rays(cb, W: int, H: int, px, py, ox: float = 0.5, oy: float = 0.5) -> np.ndarray:
    """RayGen's float32 camera rays (the frame's exact bits) for pixels (px, py): (n, 8) float32 rows
    (o.xyz, tmin 0, d.xyz, tmax 1e5), the trace_rays layout."""
    c, cp = _f(cb)
    x = np.ascontiguousarray(px, dtype=np.uint32)
    y = np.ascontiguousarray(py, dtype=np.uint32)
    out = np.zeros((x.size, 8), np.float32)
    lib.oracle_camera_rays(cp, W, H, x.ctypes.data_as(_P), y.ctypes.data_as(_P), x.size, ox, oy,
                           out.ctypes.data_as(_P))
    return out


def max_stack_reached(reset: bool = True) -> int:
    """Deepest per-ray (LANE-order) traversal stack the oracle reached since the last reset."""
    return int(lib.oracle_max_stack_reached(1 if reset else 0))


def pow_(x: float, y: float) -> float:
    return float(lib.oracle_pow(x, y))


class Scene:
    """Oracle twin of a product scene (same LBVH, same traversal order)."""

    def __init__(self, spec=None, library=None):
        self._lib = library if library is not None else lib
        self._h = self._lib.oracle_scene_create()
        self.blas_ids = []
        if spec is not None:
            self.load(spec)

    def __del__(self):
        if getattr(self, "_h", None) and getattr(self, "_lib", None) is not None:
            self._lib.oracle_scene_destroy(self._h)
            self._h = None

    def add_blas(self, verts, idx=None) -> int:
        v, vp = _f(verts)
        if idx is None:
            r = self._lib.oracle_add_blas(self._h, vp, v.shape[0], None, 0)
        else:
            i = np.ascontiguousarray(idx, dtype=np.uint32)
            r = self._lib.oracle_add_blas(self._h, vp, v.shape[0], i.ctypes.data_as(_P), i.size)
        if r < 0:
            raise RuntimeError("oracle_add_blas failed")
        return r

    def set_instances(self, instances):
        arr = (oracle_instance * len(instances))()
        for k, (b, x, iid, hg) in enumerate(instances):
            arr[k].blas = b
            arr[k].xform[:] = [float(v) for v in np.asarray(x, np.float32).ravel()]
            arr[k].instance_id = iid
            arr[k].hit_group = hg
        if self._lib.oracle_set_instances(self._h, arr, len(instances)):
            raise RuntimeError("oracle_set_instances failed")

    def load(self, spec):
        self.spec = spec
        self.blas_ids = [self.add_blas(v, i) for (v, i) in spec.meshes]
        self.set_instances([(self.blas_ids[m], x, iid, hg) for (m, x, iid, hg) in spec.instances])

    def blas_info(self, b):
        out = np.zeros(4, np.uint32)
        self._lib.oracle_blas_info(self._h, b, out.ctypes.data_as(_P))
        return out

    def tlas_info(self):
        out = np.zeros(4, np.uint32)
        self._lib.oracle_tlas_info(self._h, out.ctypes.data_as(_P))
        return out

    def export_blas(self, b):
        prims, nn, _, _ = self.blas_info(b)
        nodes = np.zeros(nn * 32, np.uint32)  # 128-B 4-wide nodes
        tris = np.zeros(prims * 12, np.uint32)
        self._lib.oracle_export_blas(self._h, b, nodes.ctypes.data_as(_P), tris.ctypes.data_as(_P))
        return nodes.reshape(-1, 32), tris.reshape(-1, 12)

    def export_tlas(self):
        _, nn, _, _ = self.tlas_info()
        nodes = np.zeros(nn * 32, np.uint32)
        self._lib.oracle_export_tlas(self._h, nodes.ctypes.data_as(_P))
        return nodes.reshape(-1, 32)

    def render(self, cb, lights, material, mode, spp, W, H, rows: Optional[np.ndarray] = None, nthreads=1,
               brute_force=False, want_float=True, schedule=0, split=0):
        """split (packet schedule): the device's forced tile-balance layouts (rt_set_tile_balance(2 + split - 1)):
        1 every tile in 2 x 2 parts, 2 in 4 x 4, 3 by tile position; each part traced as its own packet."""
        c, cp = _f(cb)
        m, mp = _f(material)
        nrows = H if rows is None else len(rows)
        rgba8 = np.zeros((nrows, W, 4), np.uint8)
        rgba32 = np.zeros((nrows, W, 4), np.float32) if want_float else None
        stats = np.zeros(12, np.uint64)
        rp = None
        if rows is not None:
            r = np.ascontiguousarray(rows, dtype=np.uint32)
            rp = r.ctypes.data_as(_P)
        st = self._lib.oracle_render_split(self._h, cp, _lights(lights), len(lights), mp, mode, spp, W, H, rp, nrows,
                                           rgba8.ctypes.data_as(_P), rgba32.ctypes.data_as(_P) if want_float else None,
                                           nthreads, stats.ctypes.data_as(_P), 1 if brute_force else 0, schedule, split)
        if st:
            raise RuntimeError("oracle_render failed")
        return rgba8, rgba32, stats

    def render_spec(self, spec, rows=None, nthreads=1, brute_force=False, want_float=True, schedule=0, split=0):
        return self.render(spec.camera_buffer(), spec.lights, spec.material, spec.mode, spec.spp, spec.width,
                           spec.height, rows, nthreads, brute_force, want_float, schedule, split)

    def trace_rays(self, rays: np.ndarray, any_hit=False, brute_force=False, cull_back=False, cull_front=False):
        r = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 8)
        n = r.shape[0]
        hits = np.zeros((n, 4), np.uint32)
        uv = np.zeros((n, 2), np.float32)
        stats = np.zeros(12, np.uint64)
        flags = (0x04 if any_hit else 0) | (0x10 if cull_back else 0) | (0x20 if cull_front else 0)  # D3D12_RAY_FLAG
        if self._lib.oracle_trace_rays(self._h, r.ctypes.data_as(_P), n, flags, hits.ctypes.data_as(_P),
                              uv.ctypes.data_as(_P), 1 if brute_force else 0, stats.ctypes.data_as(_P)):
            raise RuntimeError("oracle_trace_rays failed")
        return hits, uv, stats
