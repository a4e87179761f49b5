"""Seeded random scenes for the parity tests (test helper, not part of the package).

Each seed draws: 1..3 meshes (non-indexed triangle soups of clustered, sliver and axis-aligned triangles, indexed
random meshes over a shared vertex pool, sometimes the teapot or the rabbit), 1..24 instances of them under random
rotations, non-uniform scales (some mirrored) and translations, with the model or the plane hit group, the ground
plane, 1..6 lights, a random material (reflective for InstanceID 0 and 1 in REF mode when reflectivity > 0), a
random camera aimed at the scene, one of the three shading modes and 1 or 4 samples per pixel (LAMBERT_SHADOW).
Vertex normals are the face normal plus noise, normalised (as ComputeVertexNormals leaves them unit length).
"""
import numpy as np

from realtimeraytracing_gradproject_amd import (RT_HITGROUP_MODEL, RT_HITGROUP_PLANE, RT_SHADE_LAMBERT_SHADOW,
                                                RT_SHADE_PRIMARY, RT_SHADE_REF, plane_vertices)
from realtimeraytracing_gradproject_amd import scenes


def _with_normals(p, rng):
    """p: (ntri, 3, 3) positions -> (3 ntri, 6) vertices with noisy unit normals."""
    e1, e2 = p[:, 1] - p[:, 0], p[:, 2] - p[:, 0]
    fn = np.cross(e1, e2)
    ln = np.linalg.norm(fn, axis=1, keepdims=True)
    fn = np.where(ln > 0, fn / np.maximum(ln, 1e-30), [0.0, 1.0, 0.0])
    n = fn[:, None, :] + rng.normal(scale=0.3, size=(p.shape[0], 3, 3))
    n /= np.maximum(np.linalg.norm(n, axis=2, keepdims=True), 1e-6)
    out = np.zeros((p.shape[0] * 3, 6), np.float32)
    out[:, :3] = p.reshape(-1, 3)
    out[:, 3:] = n.reshape(-1, 3)
    return out


def random_soup(rng, ntri):
    """Clusters of small triangles, a few slivers across the cluster and a few axis-aligned (zero-thickness) ones."""
    ncl = int(rng.integers(1, 6))
    cent = rng.uniform(-2.0, 2.0, size=(ncl, 3))
    which = rng.integers(0, ncl, size=ntri)
    size = rng.choice([0.05, 0.2, 0.6], size=ntri)
    p = cent[which][:, None, :] + rng.normal(size=(ntri, 3, 3)) * size[:, None, None]
    kind = rng.integers(0, 10, size=ntri)
    sl = kind == 0
    p[sl, 1] = -p[sl, 0] + rng.normal(scale=1e-3, size=(int(sl.sum()), 3))
    fl = kind == 1
    p[fl, :, 1] = p[fl, :1, 1]
    return _with_normals(p.astype(np.float64), rng), None


def random_indexed(rng, ntri):
    """A shared pool of vertices on a bumpy sheet and random index triples (some repeated, some degenerate)."""
    nv = int(max(3, ntri // 2))
    u = rng.uniform(-2, 2, size=(nv, 2))
    pos = np.stack([u[:, 0], 0.3 * np.sin(2 * u[:, 0]) * np.cos(3 * u[:, 1]), u[:, 1]], axis=1)
    idx = rng.integers(0, nv, size=(ntri, 3)).astype(np.uint32)
    v = np.zeros((nv, 6), np.float32)
    v[:, :3] = pos
    nrm = np.stack([-0.6 * np.cos(2 * u[:, 0]) * np.cos(3 * u[:, 1]), np.ones(nv),
                    0.9 * np.sin(2 * u[:, 0]) * np.sin(3 * u[:, 1])], axis=1) + rng.normal(scale=0.2, size=(nv, 3))
    v[:, 3:] = nrm / np.linalg.norm(nrm, axis=1, keepdims=True)
    return v, idx.ravel()


def random_scene(seed, width=96, height=64, max_tris=2500, models=True):
    rng = np.random.default_rng(seed)
    meshes = []
    for _ in range(int(rng.integers(1, 4))):
        r = rng.random()
        if models and r < 0.2:
            meshes.append(scenes._model("teapot" if rng.random() < 0.5 else "rabbit"))
        elif r < 0.6:
            meshes.append(random_soup(rng, int(rng.integers(1, max_tris))))
        else:
            meshes.append(random_indexed(rng, int(rng.integers(1, max_tris))))
    meshes.append((plane_vertices(), None))
    plane = len(meshes) - 1
    inst = []
    for k in range(int(rng.integers(1, 25))):
        m = int(rng.integers(0, plane))
        scale = rng.uniform(0.3, 2.0, size=3) * np.where(rng.random(3) < 0.15, -1.0, 1.0)
        if rng.random() < 0.4:  # pure translation (the kernel's translate-only instance path)
            x = scenes.translation(*(float(t) for t in rng.uniform(-8, 8, size=3)))
        else:
            x = scenes._rot_scale(rng.normal(size=3) + 1e-3, float(rng.uniform(0, 360)), scale,
                                  rng.uniform(-8, 8, size=3))
        hg = RT_HITGROUP_PLANE if rng.random() < 0.15 else RT_HITGROUP_MODEL
        inst.append((m, x, len(inst), hg))
    inst.append((plane, scenes.IDENTITY, len(inst), RT_HITGROUP_PLANE))
    lights = [(tuple(float(c) for c in rng.uniform(0.2, 1.0, 3)), tuple(float(c) for c in rng.uniform(-12, 12, 3)),
               float(rng.uniform(0.1, 1.0))) for _ in range(int(rng.integers(1, 7)))]
    material = tuple(float(c) for c in rng.uniform(0.2, 1.0, 3)) + (float(rng.uniform(0.05, 1.0)),
                                                                     float(rng.uniform(0.0, 1.0)),
                                                                     float(rng.choice([0.0, 0.5])))
    target = rng.uniform(-3, 3, size=3)
    d = rng.normal(size=3)
    eye = target + d / np.linalg.norm(d) * float(rng.choice([3.0, 8.0, 16.0, 30.0]))
    camera = (tuple(float(c) for c in eye), tuple(float(c) for c in target), (0.0, 1.0, 0.0))
    mode = int(rng.choice([RT_SHADE_LAMBERT_SHADOW, RT_SHADE_REF, RT_SHADE_PRIMARY]))
    spp = int(rng.choice([1, 4])) if mode == RT_SHADE_LAMBERT_SHADOW else 1
    return scenes.SceneSpec(f"RND{seed}", meshes, inst, lights, material, camera, width, height, mode, spp)
