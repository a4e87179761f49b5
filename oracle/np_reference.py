"""Independent float64 numpy restatement of the reference path (test infrastructure only).

Used to cross-check the C oracle (oracle/rt_oracle.c) where the reference itself cannot run
(HLSL/DXR). It shares no code with either the oracle or the product: brute-force ray/triangle tests
over every triangle of every instance (no BVH), shading formulas transcribed from the HLSL:
  RayGen.hlsl:28-43, Common.hlsl:44-82, Hit.hlsl:67-241, Miss.hlsl:3-10, ShadowRay.hlsl:10-20,
including the ReflectRay chains of InstanceID 0 / 1 (Hit.hlsl:176-203, CastReflectionRay
Common.hlsl:58-69) evaluated as HLSL nests them: color_k = lerp(s_k, color_{k+1}, r), innermost
first, and the spp average (2x2 stratified samples).
Evaluation is float64, so agreement with the float32 oracle is to a tolerance, and pixels whose
primary ray grazes an edge can legitimately flip between triangles or between hit and miss.
"""
from __future__ import annotations

import numpy as np

PI = 3.14159265359
MAX_REFLECT = 18  # reflection rays per camera ray: 20 TraceRay levels (D3D12HelloTriangle.cpp:954), SURVEY A.6-1


def _norm(v):
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def camera_rays(cb: np.ndarray, W: int, H: int, px: np.ndarray, py: np.ndarray, ox=0.5, oy=0.5):
    cb = cb.astype(np.float64)
    view_inv = cb[32:48].reshape(4, 4).T  # HLSL reads XMMATRIX memory column-major
    proj_inv = cb[48:64].reshape(4, 4).T
    dx = ((px + ox) / W) * 2.0 - 1.0
    dy = ((py + oy) / H) * 2.0 - 1.0
    ndc = np.stack([dx, -dy, np.ones_like(dx), np.ones_like(dx)], axis=-1)
    dcam = ndc @ proj_inv.T
    dcam[:, 3] = 0.0
    d = (dcam @ view_inv.T)[:, :3]
    o = np.broadcast_to(view_inv[:3, 3], d.shape).copy()
    return o, _norm(d)


class Scene:
    def __init__(self, spec):
        self.spec = spec
        self.inst = []
        for (m, x, iid, hg) in spec.instances:
            v, idx = spec.meshes[m]
            v = np.asarray(v, np.float64)
            tri = idx.reshape(-1, 3) if idx is not None else np.arange(v.shape[0]).reshape(-1, 3)
            M = np.asarray(x, np.float64).reshape(3, 4)
            L, t = M[:, :3], M[:, 3]
            Li = np.linalg.inv(L)
            # a mirroring transform flips the front face (DXR: clockwise seen from the ray origin)
            self.inst.append(dict(v=v, tri=tri, w2o_L=Li, w2o_t=-Li @ t, nrm=Li.T, hg=hg, iid=iid,
                                  face=-1.0 if np.linalg.det(L) < 0 else 1.0))

    CHUNK = 32  # triangles per culling box (consecutive primitive indices)

    def _chunks(self, I):
        """Per-instance culling boxes over runs of CHUNK consecutive triangles (a speed-up only: no
        hierarchy, no shared code with the BVH builders); the last run is padded with det = 0
        triangles that never hit."""
        if "cp0" not in I:
            C = self.CHUNK
            p0 = I["v"][I["tri"][:, 0], :3]
            e1 = I["v"][I["tri"][:, 1], :3] - p0
            e2 = I["v"][I["tri"][:, 2], :3] - p0
            n = p0.shape[0]
            m = -(-n // C) * C
            pad = lambda a: np.concatenate([a, np.zeros((m - n, 3))]) if m > n else a
            I["cp0"], I["ce1"], I["ce2"] = pad(p0).reshape(-1, C, 3), pad(e1).reshape(-1, C, 3), pad(e2).reshape(-1, C, 3)
            pts = np.stack([p0, p0 + e1, p0 + e2], 1)
            pts = np.concatenate([pts, np.repeat(pts[-1:], m - n, 0)]) if m > n else pts
            pts = pts.reshape(-1, C * 3, 3)
            I["clo"], I["chi"] = pts.min(1) - 1e-4, pts.max(1) + 1e-4
            I["ntri"] = n
        return I

    def intersect(self, O, D, tmin, tmax, any_hit=False, cull_back=False):
        """Closest hit over every triangle of every instance: the lexicographic minimum of
        (t, instance, primitive), as DXR's closest hit with the pinned tie rule."""
        n = O.shape[0]
        best_t = np.full(n, tmax, np.float64) if np.ndim(tmax) == 0 else tmax.astype(np.float64).copy()
        best_i = np.full(n, -1, np.int64)
        best_p = np.full(n, -1, np.int64)
        bu = np.zeros(n)
        bv = np.zeros(n)
        C = self.CHUNK
        for k, I in enumerate(self.inst):
            I = self._chunks(I)
            o_all = O @ I["w2o_L"].T + I["w2o_t"]
            d_all = D @ I["w2o_L"].T
            with np.errstate(divide="ignore", invalid="ignore"):
                inv_d = 1.0 / d_all
            # (ray, run) pairs whose segment meets the run's box
            rows = []
            for s0 in range(0, n, 2048):
                o, iv = o_all[s0:s0 + 2048, None, :], inv_d[s0:s0 + 2048, None, :]
                with np.errstate(divide="ignore", invalid="ignore"):
                    ta, tb = (I["clo"][None] - o) * iv, (I["chi"][None] - o) * iv
                tn = np.nanmax(np.minimum(ta, tb), axis=2)
                tf = np.nanmin(np.maximum(ta, tb), axis=2)
                r, c = np.nonzero((tn <= tf) & (tf >= tmin) & (tn <= best_t[s0:s0 + 2048, None]))
                rows.append((r + s0, c))
            ri = np.concatenate([a for a, _ in rows])
            ci = np.concatenate([b for _, b in rows])
            for q0 in range(0, ri.size, 4096):
                rr, cc = ri[q0:q0 + 4096], ci[q0:q0 + 4096]
                oo, dd = o_all[rr][:, None, :], d_all[rr][:, None, :]
                p0, e1, e2 = I["cp0"][cc], I["ce1"][cc], I["ce2"][cc]
                pv = np.cross(dd, e2)
                det = np.sum(e1 * pv, -1)
                with np.errstate(divide="ignore", invalid="ignore"):
                    inv = 1.0 / det
                    sv = oo - p0
                    u = np.sum(sv * pv, -1) * inv
                    qv = np.cross(sv, e1)
                    v = np.sum(dd * qv, -1) * inv
                    t = np.sum(e2 * qv, -1) * inv
                ok = (det != 0) & (u >= 0) & (u <= 1) & (v >= 0) & (u + v <= 1) & (t >= tmin)
                if cull_back:  # RAY_FLAG_CULL_BACK_FACING_TRIANGLES: keep front faces only
                    ok &= det * I["face"] > 0
                t = np.where(ok, t, np.inf)
                j = np.argmin(t, axis=1)  # lowest primitive of the run on ties
                a = np.arange(rr.size)
                tj, pj = t[a, j], cc * C + j
                # per ray: smallest t, then lowest primitive (runs are in primitive order)
                order = np.lexsort((pj, tj, rr))
                rr, tj, pj, uj, vj = rr[order], tj[order], pj[order], u[a, j][order], v[a, j][order]
                first = np.ones(rr.size, bool)
                first[1:] = rr[1:] != rr[:-1]
                rr, tj, pj, uj, vj = rr[first], tj[first], pj[first], uj[first], vj[first]
                # strictly smaller t, or the same t in this instance at a lower primitive (earlier
                # instances keep ties: lower instance index)
                better = (tj < best_t[rr]) | ((tj == best_t[rr]) & (best_i[rr] == k) & (pj < best_p[rr]))
                better &= np.isfinite(tj)
                rr = rr[better]
                best_t[rr], best_i[rr], best_p[rr] = tj[better], k, pj[better]
                bu[rr], bv[rr] = uj[better], vj[better]
        return best_t, best_i, best_p, bu, bv

    def _vertex_ids(self, k, prims):
        return self.inst[k]["tri"][prims]

    def shade(self, O, D, t, inst, prim, u, v, py, mode, depth=0):
        spec = self.spec
        lights = [(np.array(c, float), np.array(p, float), float(i)) for (c, p, i) in spec.lights]
        mat = np.array(spec.material, float)
        H = spec.height
        out = np.zeros((O.shape[0], 3))
        miss = inst < 0
        out[miss] = np.stack([np.zeros(miss.sum()), np.full(miss.sum(), 0.2), 0.7 - 0.3 * (py[miss] / H)], -1)
        for k, I in enumerate(self.inst):
            sel = np.where(inst == k)[0]
            if sel.size == 0:
                continue
            P = O[sel] + D[sel] * t[sel, None]
            ids = self._vertex_ids(k, prim[sel])
            if I["hg"] == 2:
                p = I["v"][:, :3]
                n = _norm(np.cross(p[ids[:, 1]] - p[ids[:, 0]], p[ids[:, 2]] - p[ids[:, 0]])) @ I["nrm"].T
                n_out = n
            else:
                N = I["v"][:, 3:6]
                uu, vv = u[sel, None], v[sel, None]
                n = _norm(N[ids[:, 1]] * uu + N[ids[:, 2]] * vv + N[ids[:, 0]] * (1 - uu - vv))
                n = _norm(n @ I["nrm"].T)
                n_out = -n
            if mode == 0 and I["hg"] == 2:
                lp = lights[0][1]
                ld = _norm(lp - P)
                shadowed = np.sum(n * ld, -1) < 0
                _, oi, _, _, _ = self.intersect(P, ld, 0.01, 100000.0)
                shadowed |= oi >= 0
                c = np.maximum(0, np.sum(n * ld, -1)) * np.where(shadowed, 0.3, 1.0)
                out[sel] = c[:, None]
            elif mode == 0:
                s = self._direct(P, n, mat[:3], lights) + self._pbr(n, O[sel], P, lights, mat)
                r = mat[5]
                if r != 0.0 and I["iid"] in (0, 1) and depth < MAX_REFLECT:
                    # ReflectRay: normalize(reflect(normalize(WorldRayDirection()), n)), normalised
                    # again by CastReflectionRay; origin offset 0.001, TMin 0.001, TMax 1000, back
                    # faces culled; the payload colour is the nested lerp
                    dn = _norm(D[sel])
                    rd = _norm(_norm(dn - 2.0 * n * np.sum(dn * n, -1, keepdims=True)))
                    ro = P + 0.001 * rd
                    tt, ii, pp, uu2, vv2 = self.intersect(ro, rd, 0.001, 1000.0, cull_back=True)
                    c_next = self.shade(ro, rd, tt, ii, pp, uu2, vv2, py[sel], mode, depth + 1)
                    s = s + r * (c_next - s)
                out[sel] = s
            else:
                c = np.zeros(sel.size)
                for (lc, lp, li) in lights:
                    L = _norm(lp - P)
                    nl = np.sum(n_out * L, -1)
                    f = np.ones(sel.size)
                    if mode == 1:
                        lit = np.where(nl > 0)[0]
                        if lit.size:
                            _, oi, _, _, _ = self.intersect(P[lit], L[lit], 0.01, 100000.0)
                            f[lit] = np.where(oi >= 0, 0.3, 1.0)
                    c += np.where(nl > 0, nl * f, 0.0)
                out[sel] = (c / len(lights))[:, None]
        return out

    @staticmethod
    def _direct(P, n, albedo, lights):
        c = np.zeros_like(P)
        for (lc, lp, li) in lights:
            tl = -_norm(lp - P)
            c += albedo * lc * np.maximum(0.0, np.sum(n * tl, -1) * li)[:, None]
        return c

    @staticmethod
    def _pbr(n, cam, P, lights, mat):
        albedo, rough, metal = mat[:3], mat[3], mat[4]
        N = -_norm(n)
        V = _norm(cam - P)
        L0 = np.zeros_like(P)
        for (lc, lp, li) in lights:
            L = _norm(lp - P)
            Hh = _norm(V + L)
            dist = np.linalg.norm(lp - P, axis=-1)
            att = 1.0 / np.maximum(dist * dist, 1.0)
            rad = lc * att[:, None]
            F0 = 0.04 + metal * (albedo - 0.04)
            x = np.clip(1.0 - np.maximum(np.sum(Hh * V, -1), 0.0), 0, 1)
            F = F0 + (1 - F0) * (x ** 5)[:, None]
            a2 = (rough * rough) ** 2
            ndh = np.maximum(np.sum(N * Hh, -1), 0)
            den = ndh * ndh * (a2 - 1) + 1
            NDF = a2 / (PI * den * den)
            k = (rough + 1) ** 2 / 8
            ndv = np.maximum(np.sum(N * V, -1), 0)
            ndl = np.maximum(np.sum(N * L, -1), 0)
            G = (ndl / (ndl * (1 - k) + k)) * (ndv / (ndv * (1 - k) + k))
            spec = (NDF * G)[:, None] * F / (4 * ndv * ndl + 0.0001)[:, None]
            kD = (1 - F) * (1 - metal)
            L0 += (kD * albedo / PI + spec) * rad * ndl[:, None]
        c = L0 * 0.2
        c = c / (c + 1)
        return c ** (1 / 2.2)

    def render(self, cb: np.ndarray):
        spec = self.spec
        W, H = spec.width, spec.height
        k = int(round(spec.spp ** 0.5))
        yy, xx = np.mgrid[0:H, 0:W]
        px, py = xx.ravel().astype(float), yy.ravel().astype(float)
        acc = np.zeros((W * H, 3))
        ids = None
        for sy in range(k):
            for sx in range(k):
                O, D = camera_rays(cb, W, H, px, py, (sx + 0.5) / k, (sy + 0.5) / k)
                t, inst, prim, u, v = self.intersect(O, D, 0.0, 100000.0)
                if ids is None:
                    ids = np.stack([inst, prim], -1)
                acc += self.shade(O, D, t, inst, prim, u, v, py, spec.mode)
        acc /= k * k
        return acc.reshape(H, W, 3), ids.reshape(H, W, 2)
