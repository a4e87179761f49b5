/*
 * rt_raster_oracle.c — CPU ORACLE (test infrastructure, not product code) for the raster
 * fallback (rt_raster_draw). Used only by tests/ as the checker.
 *
 * Restates the reference's abandoned rasterization pipeline (shaders/shaders.hlsl:41-59 VSMain /
 * PSMain, draws recorded at D3D12HelloTriangle.cpp:513-540, pipeline state :248-276, depth buffer
 * :1340-1360) under the Direct3D rasterization rules, processed the way the API defines them:
 * draw after draw, triangle after triangle, every covered pixel depth-tested LESS against a D32
 * buffer cleared to 1.0 and written in submission order. (The device reaches the same image
 * order-independently — per-pixel minimum of (depth, primitive) over tile bins filled in arbitrary
 * order; this in-order form is what proves that equivalence.)
 *
 * Pinned rules: clip 0 <= z <= w plus a |x|,|y| <= 4w guard band (Sutherland-Hodgman,
 * the inside vertex as the interpolation origin), viewport X = (x/w + 1) W/2, Y = (1 - y/w) H/2,
 * 16.8 fixed-point snap (round half to even), pixel centres at +0.5, front = clockwise on screen
 * (FrontCounterClockwise = FALSE, CullMode BACK), top-left fill rule, depth linear in screen
 * space clamped to [0, 1], COLOR perspective-correct from the homogeneous vertices. COLOR is the
 * R32G32B32A32 element at byte 12 of the 24-byte Vertex (:253-257): normal.xyz and the next
 * vertex's position.x, all zero for the last vertex (out-of-bounds fetch).
 *
 * Parity unpinned against reference execution (D3D12 only): restated from the source text and
 * the D3D rules; cross-checked in tests against the ray tracer's primary hits traced with
 * RAY_FLAG_CULL_FRONT_FACING_TRIANGLES (tests/test_raster.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "rt_oracle.h"

typedef struct {
  float x, y, z, w;
} rv4;

/* HLSL mul(M, v), M read column-major from XMMATRIX memory (matches the RayGen restatement) */
static void rmul4(const float* m, const float v[4], float r[4]) {
  for (int i = 0; i < 4; ++i) r[i] = ((m[i] * v[0] + m[4 + i] * v[1]) + m[8 + i] * v[2]) + m[12 + i] * v[3];
}

static float rplane(rv4 v, int p) {
  switch (p) {
    case 0: return v.z;
    case 1: return v.w - v.z;
    case 2: return v.x + 4.0f * v.w;
    case 3: return 4.0f * v.w - v.x;
    case 4: return v.y + 4.0f * v.w;
    default: return 4.0f * v.w - v.y;
  }
}

static rv4 rlerp(rv4 in, float din, rv4 out, float dout) {
  const float t = din / (din - dout);
  rv4 r = {in.x + t * (out.x - in.x), in.y + t * (out.y - in.y), in.z + t * (out.z - in.z), in.w + t * (out.w - in.w)};
  return r;
}

static int64_t rfloordiv(int64_t a, int64_t b) {
  int64_t q = a / b;
  if (a % b != 0 && a < 0) q -= 1;
  return q;
}

static uint32_t rnorm8(float c) {
  if (!(c > 0.0f)) return 0u;
  if (c >= 1.0f) return 255u;
  return (uint32_t)(c * 255.0f + 0.5f);
}

int oracle_raster(const float* const* vtx6, const uint32_t* nvtx, const uint32_t* const* idx, const uint32_t* ntri,
                  uint32_t ndraws, const float o2w3x4[12], const float cb[64], uint32_t W, uint32_t H,
                  uint8_t* rgba8, float* depth_out, uint32_t* prim_out) {
  if (!W || !H || ndraws == 0) return -1;
  /* instance objectToWorld as XMMATRIX memory: memory row j = column j of the 3x4 transform */
  float xm[16];
  for (int j = 0; j < 4; ++j) {
    for (int i = 0; i < 3; ++i) xm[j * 4 + i] = o2w3x4[i * 4 + j];
    xm[j * 4 + 3] = j == 3 ? 1.0f : 0.0f;
  }
  const size_t npx = (size_t)W * H;
  float* depth = (float*)malloc(npx * sizeof(float));
  uint32_t* prim = (uint32_t*)malloc(npx * sizeof(uint32_t));
  uint64_t ntot = 0;
  for (uint32_t d = 0; d < ndraws; ++d) ntot += ntri[d];
  rv4* clip = (rv4*)malloc((size_t)(ntot ? ntot : 1) * 3 * sizeof(rv4));
  if (!depth || !prim || !clip) {
    free(depth);
    free(prim);
    free(clip);
    return -2;
  }
  for (size_t p = 0; p < npx; ++p) {
    depth[p] = 1.0f; /* ClearDepthStencilView(1.0) */
    prim[p] = 0xffffffffu;
  }
  uint32_t id = 0;
  for (uint32_t d = 0; d < ndraws; ++d) {
    for (uint32_t t = 0; t < ntri[d]; ++t, ++id) {
      rv4 v[3];
      for (int k = 0; k < 3; ++k) {
        const uint32_t vi = idx[d] ? idx[d][t * 3 + k] : t * 3 + k;
        const float pos[4] = {vtx6[d][vi * 6 + 0], vtx6[d][vi * 6 + 1], vtx6[d][vi * 6 + 2], 1.0f};
        float w4[4], e4[4], c4[4];
        rmul4(xm, pos, w4);     /* objectToWorld */
        rmul4(cb, w4, e4);      /* view */
        rmul4(cb + 16, e4, c4); /* projection */
        v[k].x = c4[0], v[k].y = c4[1], v[k].z = c4[2], v[k].w = c4[3];
        clip[(size_t)id * 3 + k] = v[k];
      }
      rv4 poly[9], nxt[9];
      int n = 3;
      for (int k = 0; k < 3; ++k) poly[k] = v[k];
      for (int p = 0; p < 6 && n > 0; ++p) {
        int inside = 1;
        for (int k = 0; k < n; ++k)
          if (!(rplane(poly[k], p) >= 0.0f)) inside = 0;
        if (inside) continue;
        int m = 0;
        for (int k = 0; k < n; ++k) {
          const rv4 a = poly[k], b = poly[(k + 1) % n];
          const float da = rplane(a, p), db = rplane(b, p);
          const int ain = da >= 0.0f, bin = db >= 0.0f;
          if (ain) nxt[m++] = a;
          if (ain != bin) nxt[m++] = ain ? rlerp(a, da, b, db) : rlerp(b, db, a, da);
        }
        n = m;
        memcpy(poly, nxt, sizeof(rv4) * (size_t)n);
      }
      if (n < 3) continue;
      int32_t X[9], Y[9];
      float Z[9];
      int bad = 0;
      for (int k = 0; k < n; ++k) {
        if (!(poly[k].w > 0.0f)) bad = 1;
        const float sx = (poly[k].x / poly[k].w + 1.0f) * (0.5f * (float)W);
        const float sy = (1.0f - poly[k].y / poly[k].w) * (0.5f * (float)H);
        X[k] = (int32_t)rintf(sx * 256.0f);
        Y[k] = (int32_t)rintf(sy * 256.0f);
        Z[k] = poly[k].z / poly[k].w + 0.0f;
      }
      if (bad) continue;
      for (int f = 0; f + 2 < n; ++f) { /* fan from vertex 0 */
        const int32_t tx[3] = {X[0], X[f + 1], X[f + 2]}, ty[3] = {Y[0], Y[f + 1], Y[f + 2]};
        const float tz[3] = {Z[0], Z[f + 1], Z[f + 2]};
        const int64_t area = (int64_t)(tx[1] - tx[0]) * (ty[2] - ty[0]) - (int64_t)(ty[1] - ty[0]) * (tx[2] - tx[0]);
        if (area <= 0) continue; /* counter-clockwise (back) or degenerate */
        int32_t xmin = tx[0], xmax = tx[0], ymin = ty[0], ymax = ty[0];
        for (int k = 1; k < 3; ++k) {
          xmin = tx[k] < xmin ? tx[k] : xmin;
          xmax = tx[k] > xmax ? tx[k] : xmax;
          ymin = ty[k] < ymin ? ty[k] : ymin;
          ymax = ty[k] > ymax ? ty[k] : ymax;
        }
        int64_t x0 = -rfloordiv(128 - (int64_t)xmin, 256), x1 = rfloordiv((int64_t)xmax - 128, 256);
        int64_t y0 = -rfloordiv(128 - (int64_t)ymin, 256), y1 = rfloordiv((int64_t)ymax - 128, 256);
        if (x0 < 0) x0 = 0;
        if (y0 < 0) y0 = 0;
        if (x1 > (int64_t)W - 1) x1 = (int64_t)W - 1;
        if (y1 > (int64_t)H - 1) y1 = (int64_t)H - 1;
        for (int64_t py = y0; py <= y1; ++py)
          for (int64_t px = x0; px <= x1; ++px) {
            const int64_t cx = px * 256 + 128, cy = py * 256 + 128;
            int64_t e[3];
            int covered = 1;
            for (int i = 0; i < 3; ++i) {
              const int a = (i + 1) % 3, b = (i + 2) % 3;
              const int64_t dx = (int64_t)tx[b] - tx[a], dy = (int64_t)ty[b] - ty[a];
              e[i] = dx * (cy - ty[a]) - dy * (cx - tx[a]);
              const int top_left = dy < 0 || (dy == 0 && dx > 0);
              if (!(e[i] > 0 || (e[i] == 0 && top_left))) covered = 0;
            }
            if (!covered) continue;
            /* depth linear in screen space: z0 + (E1 (z1 - z0) + E2 (z2 - z0)) / area, in double */
            const double A = (double)(e[0] + e[1] + e[2]);
            const double dz = ((double)e[1] * ((double)tz[1] - (double)tz[0]) + (double)e[2] * ((double)tz[2] - (double)tz[0])) / A;
            float z = (float)((double)tz[0] + dz);
            if (z < 0.0f) z = 0.0f;
            const size_t o = (size_t)py * W + (size_t)px;
            if (z < depth[o]) { /* DepthFunc LESS, in submission order */
              depth[o] = z;
              prim[o] = id;
            }
          }
      }
    }
  }
  /* PSMain: interpolated COLOR */
  for (uint32_t y = 0; y < H; ++y)
    for (uint32_t x = 0; x < W; ++x) {
      const size_t o = (size_t)y * W + x;
      uint8_t* px = rgba8 + o * 4;
      if (prim_out) prim_out[o] = prim[o];
      if (depth_out) depth_out[o] = prim[o] == 0xffffffffu ? 1.0f : depth[o] + 0.0f;
      if (prim[o] == 0xffffffffu) { /* ClearRenderTargetView {0.03, 0.35, 0.43, 1} */
        px[0] = (uint8_t)rnorm8(0.03f), px[1] = (uint8_t)rnorm8(0.35f), px[2] = (uint8_t)rnorm8(0.43f);
        px[3] = (uint8_t)rnorm8(1.0f);
        continue;
      }
      uint32_t t = prim[o], d = 0;
      while (t >= ntri[d]) t -= ntri[d++];
      float col[3][4];
      for (int k = 0; k < 3; ++k) {
        const uint32_t vi = idx[d] ? idx[d][t * 3 + k] : t * 3 + k;
        const int in = vi + 1 < nvtx[d];
        for (int c = 0; c < 3; ++c) col[k][c] = in ? vtx6[d][vi * 6 + 3 + c] : 0.0f;
        col[k][3] = in ? vtx6[d][(vi + 1) * 6] : 0.0f;
      }
      const rv4* cv = clip + (size_t)prim[o] * 3;
      const float qx = (((float)x + 0.5f) / (float)W) * 2.0f - 1.0f;
      const float qy = 1.0f - (((float)y + 0.5f) / (float)H) * 2.0f;
      float f[3];
      for (int k = 0; k < 3; ++k) {
        const rv4 a = cv[(k + 1) % 3], b = cv[(k + 2) % 3];
        /* cross((a.x, a.y, a.w), (b.x, b.y, b.w)) . (qx, qy, 1) */
        const float cxx = a.y * b.w - a.w * b.y, cyy = a.w * b.x - a.x * b.w, czz = a.x * b.y - a.y * b.x;
        f[k] = (cxx * qx + cyy * qy) + czz * 1.0f;
      }
      const float sum = (f[0] + f[1]) + f[2];
      const float b0 = f[0] / sum, b1 = f[1] / sum, b2 = f[2] / sum;
      for (int c = 0; c < 4; ++c) px[c] = (uint8_t)rnorm8((b0 * col[0][c] + b1 * col[1][c]) + b2 * col[2][c]);
    }
  free(depth);
  free(prim);
  free(clip);
  return 0;
}
