"""Scene descriptions: the reference scene and the BASELINE configs C1..C5.

Reference scene (D3D12HelloTriangle::CreateAccelerationStructures, D3D12HelloTriangle.cpp:778-810):
teapot.obj with vertex normals (:335-346), 6 model instances (identity, (-5,0,5) twice, (-5,0,-5),
(5,0,-5), (5,0,5)) with hit group 0 and the ground plane (CreatePlaneVB :1237-1271) with hit group 2;
InstanceID = list index (:749). Lights: Hit.hlsl:48-57. Material: UIConstructor defaults
(UIConstructor.cpp:13-17) with reflectivity pinned to 0. Camera: setLookat((1.5,1.5,1.5),
(0,0,0), (0,1,0)) (D3D12HelloTriangle.cpp:45), 45 deg, near 0.1, far 1000 (:1154-1156), 1280x720
(Main.cpp:18).

BASELINE configs: C1 teapot 512^2 primary only; C2 teapot 1080p primary+shadow;
C3 rabbit 1080p; C4 rabbit x64 grid, 2 lights; C5 rabbit x256 grid, 4 lights, 4K, 4 spp.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np

from . import (RT_HITGROUP_MODEL, RT_HITGROUP_PLANE, RT_SHADE_LAMBERT_SHADOW, RT_SHADE_PRIMARY, RT_SHADE_REF,
               Mesh, camera_buffer, camera_lookat, plane_vertices)

# Hit.hlsl:51-56 — colour, position, intensity
REFERENCE_LIGHTS = [
    ((1.0, 1.0, 1.0), (0.0, 10.0, 0.0), 0.2),
    ((1.0, 1.0, 1.0), (10.0, 10.0, 0.0), 0.2),
    ((1.0, 1.0, 1.0), (-10.0, 10.0, 0.0), 0.2),
    ((1.0, 1.0, 1.0), (0.0, 10.0, 10.0), 0.2),
    ((1.0, 1.0, 1.0), (0.0, 10.0, -10.0), 0.2),
    ((1.0, 1.0, 1.0), (0.0, -10.0, 0.0), 0.2),
]
# albedo rgb, roughness, metallic, reflectivity (UIConstructor.cpp:13-17; reflectivity pinned 0)
REFERENCE_MATERIAL = (1.0, 1.0, 1.0, 0.5, 0.5, 0.0)
REFERENCE_CAMERA = ((1.5, 1.5, 1.5), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0))


def translation(tx: float, ty: float, tz: float) -> np.ndarray:
    return np.array([1, 0, 0, tx, 0, 1, 0, ty, 0, 0, 1, tz], np.float32)


IDENTITY = translation(0, 0, 0)


@dataclass
class SceneSpec:
    name: str
    meshes: List[Tuple[np.ndarray, Optional[np.ndarray]]]  # (vertices N x 6, indices or None)
    instances: List[Tuple[int, np.ndarray, int, int]]      # (mesh index, 3x4 xform, instance id, hit group)
    lights: list
    material: tuple
    camera: tuple
    width: int
    height: int
    mode: int
    spp: int = 1
    fov_deg: float = 45.0
    model: str = "teapot"

    def camera_buffer(self) -> np.ndarray:
        view = camera_lookat(*self.camera)
        return camera_buffer(view, self.width, self.height, self.fov_deg, 0.1, 1000.0)

    def with_size(self, width: int, height: int) -> "SceneSpec":
        s = SceneSpec(**{**self.__dict__})
        s.width, s.height = width, height
        return s

    @property
    def triangles(self) -> int:
        return sum((m[1].size // 3 if m[1] is not None else m[0].shape[0] // 3) for m in self.meshes)


def load_model(name: str) -> Tuple[np.ndarray, np.ndarray]:
    """OBJ ingest + ComputeVertexNormals, as LoadAssets does (D3D12HelloTriangle.cpp:335-346)."""
    m = Mesh.asset(name).compute_vertex_normals()
    return m.vertices, m.indices


_model_cache = {}


def _model(name: str):
    if name not in _model_cache:
        _model_cache[name] = load_model(name)
    return _model_cache[name]


def reference_scene() -> SceneSpec:
    model = _model("teapot")
    inst = [
        (0, translation(0, 0, 0), 0, RT_HITGROUP_MODEL),
        (0, translation(-5, 0, 5), 1, RT_HITGROUP_MODEL),
        (0, translation(-5, 0, 5), 2, RT_HITGROUP_MODEL),
        (0, translation(-5, 0, -5), 3, RT_HITGROUP_MODEL),
        (0, translation(5, 0, -5), 4, RT_HITGROUP_MODEL),
        (0, translation(5, 0, 5), 5, RT_HITGROUP_MODEL),
        (1, IDENTITY, 6, RT_HITGROUP_PLANE),
    ]
    return SceneSpec("reference", [model, (plane_vertices(), None)], inst, REFERENCE_LIGHTS,
                     REFERENCE_MATERIAL, REFERENCE_CAMERA, 1280, 720, RT_SHADE_REF)


def _single(name: str, tag: str, w: int, h: int, mode: int, nlights: int = 1) -> SceneSpec:
    model = _model(name)
    inst = [(0, IDENTITY, 0, RT_HITGROUP_MODEL), (1, IDENTITY, 1, RT_HITGROUP_PLANE)]
    return SceneSpec(tag, [model, (plane_vertices(), None)], inst, REFERENCE_LIGHTS[:nlights],
                     REFERENCE_MATERIAL, REFERENCE_CAMERA, w, h, mode, model=name)


def _grid(name: str, tag: str, side: int, nlights: int, w: int, h: int, spp: int, camera) -> SceneSpec:
    model = _model(name)
    inst = []
    half = (side - 1) / 2.0
    for i in range(side):
        for j in range(side):
            inst.append((0, translation((i - half) * 3.0, 0.0, (j - half) * 3.0), len(inst), RT_HITGROUP_MODEL))
    inst.append((1, IDENTITY, len(inst), RT_HITGROUP_PLANE))
    return SceneSpec(tag, [model, (plane_vertices(), None)], inst, REFERENCE_LIGHTS[:nlights], REFERENCE_MATERIAL,
                     camera, w, h, RT_SHADE_LAMBERT_SHADOW, spp, model=name)


def config(name: str) -> SceneSpec:
    name = name.upper()
    if name == "REF":
        return reference_scene()
    if name == "C1":
        return _single("teapot", "C1", 512, 512, RT_SHADE_PRIMARY)
    if name == "C2":
        return _single("teapot", "C2", 1920, 1080, RT_SHADE_LAMBERT_SHADOW)
    if name == "C2F":
        # C2 with the teapot framed from outside (the reference camera sits inside the teapot body)
        s = _single("teapot", "C2F", 1920, 1080, RT_SHADE_LAMBERT_SHADOW)
        s.camera = ((7.0, 5.0, 9.0), (0.2, 1.3, 0.0), (0.0, 1.0, 0.0))
        return s
    if name == "C3":
        return _single("rabbit", "C3", 1920, 1080, RT_SHADE_LAMBERT_SHADOW)
    if name == "C4":
        return _grid("rabbit", "C4", 8, 2, 1920, 1080, 1, ((18.0, 14.0, 18.0), (0.0, 1.0, 0.0), (0.0, 1.0, 0.0)))
    if name == "C5":
        return _grid("rabbit", "C5", 16, 4, 3840, 2160, 4, ((30.0, 22.0, 30.0), (0.0, 1.0, 0.0), (0.0, 1.0, 0.0)))
    if name in ("REFL", "REFLO"):
        # the reference scene with a reflective material (reflectivity is never
        # initialised in the reference, UIConstructor.h:41; 0.5 here): InstanceID 0 and 1 trace
        # reflection rays. REFL keeps the reference camera (inside teapot 0: long mirror chains),
        # REFLO looks at the scene from outside.
        s = reference_scene()
        s.name = name
        s.material = REFERENCE_MATERIAL[:5] + (0.5,)
        if name == "REFLO":
            s.camera = ((9.0, 6.0, 11.0), (-1.5, 0.5, 0.0), (0.0, 1.0, 0.0))
        return s
    if name == "DEGEN":
        return degenerate_scene()
    if name == "DEEP":
        return deep_scene()
    raise KeyError(name)


CONFIGS = ("REF", "C1", "C2", "C2F", "C3", "C4", "C5", "REFL", "REFLO", "DEGEN")


def _rot_scale(axis, angle_deg: float, scale, t) -> np.ndarray:
    """3x4 row-major object-to-world: rotation about `axis`, then per-axis scale, then translation."""
    a = np.asarray(axis, np.float64)
    a = a / np.linalg.norm(a)
    c, s = np.cos(np.radians(angle_deg)), np.sin(np.radians(angle_deg))
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    R = np.eye(3) + s * K + (1 - c) * (K @ K)
    M = np.diag(np.asarray(scale, np.float64)) @ R
    x = np.zeros((3, 4))
    x[:, :3] = M
    x[:, 3] = t
    return x.astype(np.float32).ravel()


def degenerate_soup(ntri: int = 1500, seed: int = 77) -> np.ndarray:
    """Non-indexed triangle soup with the inputs an LBVH build and Moller-Trumbore must survive:
    ordinary triangles, collinear (zero-area) ones, single points, exact duplicates, slivers
    spanning the whole box and axis-aligned (zero-thickness) ones. Normals (0,1,0)."""
    rng = np.random.default_rng(seed)
    p = np.empty((ntri, 3, 3), np.float32)
    kind = rng.integers(0, 6, size=ntri)
    for k in range(ntri):
        c = rng.uniform(-3.0, 3.0, size=3)
        v = c + rng.normal(scale=0.35, size=(3, 3))
        if kind[k] == 1:    # collinear
            v[2] = v[0] + rng.uniform(-2.0, 2.0) * (v[1] - v[0])
        elif kind[k] == 2:  # a point
            v[:] = v[0]
        elif kind[k] == 3 and k > 0:  # duplicate of the previous triangle
            v = p[k - 1].astype(np.float64)
        elif kind[k] == 4:  # sliver across the box
            v[1] = -v[0] + rng.normal(scale=1e-3, size=3)
            v[2] = v[1] + rng.normal(scale=1e-4, size=3)
        elif kind[k] == 5:  # zero thickness in y
            v[:, 1] = v[0, 1]
        p[k] = v
    out = np.zeros((ntri * 3, 6), np.float32)
    out[:, :3] = p.reshape(-1, 3)
    out[:, 4] = 1.0
    return out


def point_cloud_mesh(ntri: int = 16) -> np.ndarray:
    """Every vertex at one point: a BLAS whose bounds have zero extent on all three axes."""
    out = np.zeros((ntri * 3, 6), np.float32)
    out[:, :3] = (0.25, 0.5, -0.75)
    out[:, 4] = 1.0
    return out


def degenerate_scene() -> SceneSpec:
    """DEGEN: the degenerate soup under identity, rotated + non-uniformly scaled, and mirrored
    instances, the teapot rotated, a zero-extent BLAS and the ground plane (test scene, not a
    BASELINE config)."""
    teapot = _model("teapot")
    meshes = [(degenerate_soup(), None), teapot, (point_cloud_mesh(), None), (plane_vertices(), None)]
    inst = [
        (0, IDENTITY, 0, RT_HITGROUP_MODEL),
        (0, _rot_scale((1, 2, 0.5), 33.0, (1.5, 0.6, 1.0), (6.0, 1.0, -2.0)), 1, RT_HITGROUP_MODEL),
        (0, _rot_scale((0, 1, 0), -70.0, (-1.0, 1.0, 1.0), (-6.0, 2.0, 1.0)), 2, RT_HITGROUP_MODEL),  # mirrored
        (1, _rot_scale((0.3, 1, -0.2), 125.0, (1.2, 1.2, 1.2), (0.0, 0.5, 6.0)), 3, RT_HITGROUP_MODEL),
        (2, IDENTITY, 4, RT_HITGROUP_MODEL),
        (3, IDENTITY, 5, RT_HITGROUP_PLANE),
    ]
    return SceneSpec("DEGEN", meshes, inst, REFERENCE_LIGHTS[:2], REFERENCE_MATERIAL,
                     ((14.0, 9.0, 16.0), (0.0, 1.0, 1.0), (0.0, 1.0, 0.0)), 320, 180, RT_SHADE_LAMBERT_SHADOW)


def deep_chain_mesh(reps: int = 8, half: float = 60.0, seed: int = 5) -> np.ndarray:
    """A BLAS whose 4-wide tree is deeper than the trace kernels' 32-entry LDS stack, with paths that
    really use that depth: triangle box centres on a Morton chain (one axis coordinate 2^j / 1024 of
    the centre bounds, j = 9..0, per axis: the binary LBVH is a 30-level chain) and every triangle
    large (2 x `half` across, facing +z), so a ray crossing the scene enters nearly every box of a
    node and the per-lane walk pushes its siblings level after level. Test scene, not a config."""
    rng = np.random.default_rng(seed)
    cents = [np.full(3, 0.5), np.full(3, 1023.5)]  # the anchors fix the centre bounds
    for j in range(9, -1, -1):
        for ax in range(3):
            c = np.full(3, 0.5)
            c[ax] = 2 ** j + 0.5
            cents.append(c)
    tris = []
    for c in cents:
        for _ in range(reps):
            p = c / 1024.0 * 40.0 + rng.normal(scale=0.05, size=3)
            tris.append([p + (-half, -half, 0.0), p + (half, -half, 0.0), p + (0.0, half, 0.0)])
    out = np.zeros((len(tris) * 3, 6), np.float32)
    out[:, :3] = np.asarray(tris).reshape(-1, 3)
    out[:, 4] = 1.0
    return out


def deep_scene() -> SceneSpec:
    """DEEP: three instances of deep_chain_mesh (per-lane stack bound > 32: the HBM overflow stack is
    used) and the plane, LAMBERT_SHADOW, small frame (test scene for concurrent launches)."""
    m = (deep_chain_mesh(), None)
    inst = [(0, IDENTITY, 0, RT_HITGROUP_MODEL), (0, translation(3.0, 1.0, -5.0), 1, RT_HITGROUP_MODEL),
            (0, _rot_scale((0, 1, 0), 20.0, (1.0, 1.0, 1.0), (-4.0, 0.0, -9.0)), 2, RT_HITGROUP_MODEL),
            (1, IDENTITY, 3, RT_HITGROUP_PLANE)]
    return SceneSpec("DEEP", [m, (plane_vertices(), None)], inst, REFERENCE_LIGHTS[:2], REFERENCE_MATERIAL,
                     ((20.0, 22.0, 70.0), (20.0, 18.0, 0.0), (0.0, 1.0, 0.0)), 96, 64, RT_SHADE_LAMBERT_SHADOW)


def upload(ctx, spec: SceneSpec, camera: bool = True) -> List[int]:
    """Builds BLAS/TLAS and frame state of `spec` on a Context; returns the BLAS ids. camera False leaves the
    context's camera unset (launches must then bring their own: rt_dispatch_frames' camera array)."""
    ids = [ctx.blas_build(v, i) for (v, i) in spec.meshes]
    ctx.tlas_build([(ids[m], x, iid, hg) for (m, x, iid, hg) in spec.instances])
    if camera:
        ctx.set_camera(spec.camera_buffer())
    ctx.set_shading(spec.lights, spec.material, spec.mode, spec.spp)
    return ids
