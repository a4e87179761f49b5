// rt_raster.hip — raster fallback: the reference's abandoned rasterization pipeline
// (shaders/shaders.hlsl:41-59 VSMain/PSMain; D3D12HelloTriangle.cpp:513-540 draw recording;
// pipeline state :248-276) as a tile-binned rasterizer for gfx950.
//
//   1. k_raster_setup   one thread per triangle of every draw: VSMain (objectToWorld, view,
//                       projection), clip to 0 <= z <= w and a guard band, viewport transform,
//                       16.8 fixed-point snap, back-face cull (clockwise front), then up to 7 fan
//                       triangles into fixed slots 7t..7t+6 with their 8x8-pixel tile counts.
//   2. k_raster_bin<0> one wave per slot: count the 8x8 screen tiles each triangle overlaps;
//      k_raster_scan   exclusive scan of the per-tile counts -> bin offsets (the host sizes the
//                      bins from the first draw's total, later draws from the last total it read
//                      back asynchronously: no synchronisation inside a draw);
//      k_raster_bin<1> the same walk, appending the slot to each overlapped tile's bin.
//   3. k_raster_tile   one wave per screen tile, the tile's depth buffer in registers: for every
//                      binned triangle, edge functions with the top-left rule and screen-linear
//                      depth; the per-pixel minimum of (depth, primitive) is exactly in-order LESS
//                      testing (smallest depth, earliest primitive on ties) whatever the bin
//                      order. Then PSMain's interpolated COLOR (perspective-correct barycentrics
//                      of the original triangle) -> RGBA8 and depth, written once. No global
//                      atomics in the depth test.
//
// COLOR is read as the reference's input layout reads it (R32G32B32A32_FLOAT at byte 12 of a
// 24-byte Vertex, :253-257): the normal plus the next vertex's position.x; the element of the
// last vertex runs past the buffer and reads as 0 in every component (pinned: D3D returns 0 for
// an out-of-bounds input-assembler fetch).
#include "rt_internal.hpp"

namespace rt {

namespace {

constexpr float kGuard = 4.0f;  // |x|, |y| <= kGuard * w: keeps 16.8 screen coordinates in int32

struct ClipV {
  float x, y, z, w;
};

__device__ inline float plane_dist(const ClipV& v, int p) {
  switch (p) {
    case 0: return v.z;                   // near: z >= 0
    case 1: return v.w - v.z;             // far:  z <= w
    case 2: return v.x + kGuard * v.w;    // guard band
    case 3: return kGuard * v.w - v.x;
    case 4: return v.y + kGuard * v.w;
    default: return kGuard * v.w - v.y;
  }
}

// Point where the edge from the inside vertex a to the outside vertex b meets the plane.
__device__ inline ClipV clip_lerp(const ClipV& a, float da, const ClipV& b, float db) {
  const float t = da / (da - db);
  return {a.x + t * (b.x - a.x), a.y + t * (b.y - a.y), a.z + t * (b.z - a.z), a.w + t * (b.w - a.w)};
}

__device__ inline int64_t floor_div(int64_t a, int64_t b) {  // b > 0
  const int64_t q = a / b;
  return (a % b != 0 && a < 0) ? q - 1 : q;
}

__device__ inline void clip_of_vertex(const float* vtx, uint32_t v, const float* o2w_mem, const float* view,
                                      const float* proj, ClipV& out) {
  const float p[4] = {vtx[v * 6 + 0], vtx[v * 6 + 1], vtx[v * 6 + 2], 1.0f};  // POSITION, w = 1
  float wpos[4], vpos[4], c[4];
  hlsl_mul4(o2w_mem, p, wpos);  // mul(instanceProps[0].objectToWorld, position)
  hlsl_mul4(view, wpos, vpos);  // mul(view, pos)
  hlsl_mul4(proj, vpos, c);     // mul(projection, pos)
  out = {c[0], c[1], c[2], c[3]};
}

// Screen-space record of one (sub)triangle; count = its tile-box size, 0 when culled (counter-
// clockwise on screen, degenerate) or outside the viewport.
__device__ inline uint32_t make_slot(const int32_t X[3], const int32_t Y[3], const float Z[3], uint32_t prim,
                                     uint32_t width, uint32_t height, RasterSlot& r) {
  const int64_t area = (int64_t)(X[1] - X[0]) * (Y[2] - Y[0]) - (int64_t)(Y[1] - Y[0]) * (X[2] - X[0]);
  if (area <= 0) return 0;  // clockwise on screen (y down) = front face; back faces and slivers culled
  const int32_t xmin = min(X[0], min(X[1], X[2])), xmax = max(X[0], max(X[1], X[2]));
  const int32_t ymin = min(Y[0], min(Y[1], Y[2])), ymax = max(Y[0], max(Y[1], Y[2]));
  // pixels whose centre (256 px + 128) can lie inside
  int64_t px0 = -floor_div(-(int64_t)xmin + 128, 256), px1 = floor_div((int64_t)xmax - 128, 256);
  int64_t py0 = -floor_div(-(int64_t)ymin + 128, 256), py1 = floor_div((int64_t)ymax - 128, 256);
  px0 = px0 < 0 ? 0 : px0;
  py0 = py0 < 0 ? 0 : py0;
  px1 = px1 > (int64_t)width - 1 ? (int64_t)width - 1 : px1;
  py1 = py1 > (int64_t)height - 1 ? (int64_t)height - 1 : py1;
  if (px0 > px1 || py0 > py1) return 0;
  for (int k = 0; k < 3; ++k) {
    r.x[k] = X[k];
    r.y[k] = Y[k];
    r.z[k] = Z[k];
  }
  r.prim = prim;
  r.tx0 = (uint16_t)(px0 >> 3);
  r.ty0 = (uint16_t)(py0 >> 3);
  r.tw = (uint16_t)((px1 >> 3) - (px0 >> 3) + 1);
  r.th = (uint16_t)((py1 >> 3) - (py0 >> 3) + 1);
  return (uint32_t)r.tw * r.th;
}

// viewport (0, 0, W, H, 0, 1): X = (x/w + 1) W/2, Y = (1 - y/w) H/2, depth = z/w; 16.8 snap
__device__ inline void to_screen(const ClipV& v, uint32_t width, uint32_t height, int32_t& X, int32_t& Y, float& Z) {
  const float sx = (v.x / v.w + 1.0f) * (0.5f * (float)width);
  const float sy = (1.0f - v.y / v.w) * (0.5f * (float)height);
  X = (int32_t)rintf(sx * 256.0f);
  Y = (int32_t)rintf(sy * 256.0f);
  Z = v.z / v.w + 0.0f;
}

// Triangles that cross a clip plane: Sutherland-Hodgman against the 6 planes (at most 9
// vertices, the polygons in LDS so the variable-length lists are not spilled to scratch), then a
// fan from vertex 0 into slots 0..6.
constexpr int kSetupBlock = 64;

__device__ void setup_clipped(const ClipV* v, uint32_t t, uint32_t width, uint32_t height,
                              ClipV* __restrict__ poly, ClipV* __restrict__ tmp,
                              RasterSlot* __restrict__ slots, uint32_t* __restrict__ tiles) {
  int n = 3;
  for (int k = 0; k < 3; ++k) poly[k] = v[k];
  for (int p = 0; p < 6 && n > 0; ++p) {
    bool all_in = true;
    for (int k = 0; k < n; ++k) all_in = all_in && plane_dist(poly[k], p) >= 0.0f;
    if (all_in) continue;
    int m = 0;
    for (int k = 0; k < n; ++k) {
      const ClipV a = poly[k];
      const ClipV b = poly[k + 1 < n ? k + 1 : 0];
      const float da = plane_dist(a, p), db = plane_dist(b, p);
      if (da >= 0.0f) tmp[m++] = a;
      if ((da >= 0.0f) != (db >= 0.0f)) tmp[m++] = da >= 0.0f ? clip_lerp(a, da, b, db) : clip_lerp(b, db, a, da);
    }
    n = m;
    for (int k = 0; k < n; ++k) poly[k] = tmp[k];
  }
  bool ok = n >= 3;
  for (int k = 0; k < n; ++k) ok = ok && poly[k].w > 0.0f;
  for (int s = 0; s < 7; ++s) {
    const size_t slot = (size_t)t * 7 + s;
    uint32_t cnt = 0;
    if (ok && s + 2 < n) {
      int32_t X[3], Y[3];
      float Z[3];
      to_screen(poly[0], width, height, X[0], Y[0], Z[0]);
      to_screen(poly[s + 1], width, height, X[1], Y[1], Z[1]);
      to_screen(poly[s + 2], width, height, X[2], Y[2], Z[2]);
      RasterSlot r;
      cnt = make_slot(X, Y, Z, t, width, height, r);
      if (cnt) slots[slot] = r;
    }
    tiles[slot] = cnt;
  }
}

__global__ __launch_bounds__(kSetupBlock) void k_raster_setup(const RasterDraws* __restrict__ drp, uint32_t total, RasterView rv, float4* __restrict__ clip,
                                                      RasterSlot* __restrict__ slots,
                                                      uint32_t* __restrict__ tiles) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  uint32_t d = 0;
  while (d + 1 < drp->n && t >= drp->first[d + 1]) ++d;
  const uint32_t lt = t - drp->first[d];
  const float* vtx = drp->vtx[d];
  uint32_t vi[3];
  for (int k = 0; k < 3; ++k) vi[k] = drp->idx[d] ? drp->idx[d][lt * 3 + k] : lt * 3 + k;
  ClipV v[3];
  bool inside = true;
  for (int k = 0; k < 3; ++k) {
    clip_of_vertex(vtx, vi[k], rv.o2w, rv.view, rv.proj, v[k]);
    clip[(size_t)t * 3 + k] = make_float4(v[k].x, v[k].y, v[k].z, v[k].w);
    for (int p = 0; p < 6; ++p) inside = inside && plane_dist(v[k], p) >= 0.0f;
  }
  if (!inside) {
    __shared__ ClipV poly[kSetupBlock][9], tmp[kSetupBlock][9];
    setup_clipped(v, t, rv.width, rv.height, poly[threadIdx.x], tmp[threadIdx.x], slots, tiles);
    return;
  }
  // common case: no clipping needed
  const bool ok = v[0].w > 0.0f && v[1].w > 0.0f && v[2].w > 0.0f;
  int32_t X[3], Y[3];
  float Z[3];
  for (int k = 0; k < 3; ++k) to_screen(v[k], rv.width, rv.height, X[k], Y[k], Z[k]);
  RasterSlot r;
  const uint32_t cnt = ok ? make_slot(X, Y, Z, t, rv.width, rv.height, r) : 0u;
  if (cnt) slots[(size_t)t * 7] = r;
  tiles[(size_t)t * 7] = cnt;
  for (int s = 1; s < 7; ++s) tiles[(size_t)t * 7 + s] = 0;
}

// Exclusive scan of n counts into offs[0..n] (offs[n] = total) in three launches:
// k_scan_blocks scans 4096-element blocks (4 per thread, coalesced uint4 loads) and records each
// block's sum, k_scan_sums scans the block sums (one workgroup), k_scan_add adds them back.
constexpr uint32_t kScanBlock = 4096;

__device__ inline uint32_t block_exclusive(uint32_t v, uint32_t* wsum, uint32_t& total) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
  uint32_t x = v;  // inclusive scan within the wave
  for (uint32_t off = 1; off < 64u; off <<= 1) {
    const uint32_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63u) wsum[w] = x;
  __syncthreads();
  uint32_t before = 0;
  total = 0;
  for (uint32_t k = 0; k < 16u; ++k) {
    const uint32_t ws = wsum[k];
    before += k < w ? ws : 0u;
    total += ws;
  }
  __syncthreads();
  return before + x - v;
}

__global__ __launch_bounds__(1024) void k_scan_blocks(const uint32_t* __restrict__ cnt, uint32_t n,
                                                      uint32_t* __restrict__ offs, uint32_t* __restrict__ bsum) {
  __shared__ uint32_t wsum[16];
  const uint32_t i0 = blockIdx.x * kScanBlock + threadIdx.x * 4u;
  uint32_t v[4];
  for (int k = 0; k < 4; ++k) v[k] = i0 + k < n ? cnt[i0 + k] : 0u;
  const uint32_t mine = (v[0] + v[1]) + (v[2] + v[3]);
  uint32_t total;
  uint32_t run = block_exclusive(mine, wsum, total);
  for (int k = 0; k < 4; ++k) {
    if (i0 + k < n) offs[i0 + k] = run;
    run += v[k];
  }
  if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

__global__ __launch_bounds__(1024) void k_scan_sums(uint32_t* __restrict__ bsum, uint32_t nb, uint32_t n,
                                                    uint32_t* __restrict__ offs) {
  __shared__ uint32_t wsum[16];
  uint32_t carry = 0;
  for (uint32_t base = 0; base < nb; base += 1024u) {
    const uint32_t i = base + threadIdx.x;
    const uint32_t v = i < nb ? bsum[i] : 0u;
    uint32_t total;
    const uint32_t ex = block_exclusive(v, wsum, total);
    if (i < nb) bsum[i] = carry + ex;
    carry += total;
  }
  if (threadIdx.x == 0) offs[n] = carry;
}

__global__ __launch_bounds__(256) void k_scan_add(uint32_t* __restrict__ offs, uint32_t n,
                                                  const uint32_t* __restrict__ bsum) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && i >= kScanBlock) offs[i] += bsum[i / kScanBlock];
}

// Triangle-vs-tile test: false when the 8x8 tile's pixel centres all lie strictly outside one
// edge (E < 0 at the corner centre that maximises E). Conservative with respect to the fill rule.
__device__ inline bool tile_overlaps(const RasterSlot& r, uint32_t tx, uint32_t ty) {
  const int64_t x0 = (int64_t)tx * 2048 + 128, y0 = (int64_t)ty * 2048 + 128;
  for (int i = 0; i < 3; ++i) {
    const int a = (i + 1) % 3, b = (i + 2) % 3;
    const int64_t dx = (int64_t)r.x[b] - r.x[a], dy = (int64_t)r.y[b] - r.y[a];
    // E = dx (py - ya) - dy (px - xa): largest at py = max if dx > 0, px = max if dy < 0
    const int64_t py = dx > 0 ? y0 + 7 * 256 : y0, px = dy < 0 ? x0 + 7 * 256 : x0;
    if (dx * (py - r.y[a]) - dy * (px - r.x[a]) < 0) return false;
  }
  return true;
}

// Binning: one wave per slot, lanes striding over the slot's tile box. PASS 0 counts the
// overlapping (slot, tile) pairs per screen tile, PASS 1 appends the slot to the tile's bin
// (order inside a bin is arbitrary: the per-pixel minimum below does not depend on it).
template <int PASS>
__global__ __launch_bounds__(256) void k_raster_bin(const RasterSlot* __restrict__ slots,
                                                    const uint32_t* __restrict__ slot_tiles, uint32_t nslots,
                                                    uint32_t tiles_x, uint32_t* __restrict__ tcount,
                                                    const uint32_t* __restrict__ toffs, uint32_t* __restrict__ bins,
                                                    uint32_t bin_cap) {
  const uint32_t s = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (s >= nslots) return;
  const uint32_t n = slot_tiles[s];
  if (n == 0) return;
  const RasterSlot r = slots[s];
  for (uint32_t k = threadIdx.x & 63u; k < n; k += 64u) {
    const uint32_t tx = r.tx0 + k % r.tw, ty = r.ty0 + k / r.tw;
    if (!tile_overlaps(r, tx, ty)) continue;
    const uint32_t tile = ty * tiles_x + tx;
    if (PASS == 0) {
      atomicAdd(&tcount[tile], 1u);
    } else {
      // bins hold bin_cap entries: a draw with more (sized from an earlier draw's total) leaves
      // them unwritten, and k_raster_tile walks the slot list instead
      const uint32_t pos = toffs[tile] + atomicAdd(&tcount[tile], 1u);
      if (pos < bin_cap) bins[pos] = s;
    }
  }
}

// Per-pixel LESS test of one screen-space triangle (16.8 vertices X/Y, depths Z) against the
// pixel centre (px, py): edge functions with the top-left rule, screen-linear depth; keeps the
// minimum of (depth bits << 32 | primitive) in best.
__device__ __forceinline__ void raster_pixel(const int32_t (&X)[3], const int32_t (&Y)[3], const float (&Z)[3],
                                             uint32_t prim, int64_t px, int64_t py, unsigned long long& best) {
  int64_t e[3];
  bool in = true;
  for (int i = 0; i < 3; ++i) {  // E_i: edge from vertex i+1 to i+2 (opposite vertex i)
    const int a = (i + 1) % 3, c = (i + 2) % 3;
    const int64_t dx = (int64_t)X[c] - X[a], dy = (int64_t)Y[c] - Y[a];
    e[i] = dx * (py - Y[a]) - dy * (px - X[a]);
    const bool top_left = dy < 0 || (dy == 0 && dx > 0);
    in = in && (e[i] > 0 || (e[i] == 0 && top_left));
  }
  if (!in) return;
  // depth, linear in screen space: z0 + (E1 (z1 - z0) + E2 (z2 - z0)) / area, in double
  const double area = (double)(e[0] + e[1] + e[2]);
  const double dz = ((double)e[1] * ((double)Z[1] - (double)Z[0]) +
                     (double)e[2] * ((double)Z[2] - (double)Z[0])) / area;
  float z = (float)((double)Z[0] + dz);
  z = z < 0.0f ? 0.0f : z;  // viewport depth range [0, 1]
  if (!(z < 1.0f)) return;  // LESS against the 1.0 clear
  const unsigned long long key =
      ((unsigned long long)__builtin_bit_cast(uint32_t, z + 0.0f) << 32) | (unsigned long long)prim;
  best = key < best ? key : best;
}

// The triangles held by the lanes set in `live` (one slot record per lane), broadcast lane by lane.
__device__ __forceinline__ void raster_batch(uint64_t live, const int32_t (&lx)[3], const int32_t (&ly)[3],
                                             const float (&lz)[3], uint32_t lp, int64_t px, int64_t py,
                                             unsigned long long& best) {
  while (live) {
    const int j = __builtin_ctzll(live);
    live &= live - 1;
    int32_t X[3], Y[3];
    float Z[3];
    for (int k = 0; k < 3; ++k) {
      X[k] = __builtin_amdgcn_readlane(lx[k], j);
      Y[k] = __builtin_amdgcn_readlane(ly[k], j);
      Z[k] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int32_t, lz[k]), j));
    }
    raster_pixel(X, Y, Z, (uint32_t)__builtin_amdgcn_readlane((int)lp, j), px, py, best);
  }
}

// One wave per 8x8 screen tile: every binned triangle is tested against the wave's 64 pixels
// (edge functions, top-left rule, screen-linear depth); the per-pixel minimum of
// (depth bits << 32 | primitive) is exactly in-order LESS testing. The winning primitive is then
// shaded (PSMain: interpolated COLOR) and written once.
__global__ __launch_bounds__(256) void k_raster_tile(const RasterDraws* __restrict__ drp, const float4* __restrict__ clip,
                                                     const RasterSlot* __restrict__ slots,
                                                     const uint32_t* __restrict__ toffs,
                                                     const uint32_t* __restrict__ bins, uint32_t bin_cap,
                                                     const uint32_t* __restrict__ slot_tiles, uint32_t nslots,
                                                     uint32_t tiles_x, uint32_t ntiles, uint32_t width,
                                                     uint32_t height, uint32_t* __restrict__ rgba8,
                                                     float* __restrict__ depth) {
  const uint32_t tile = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (tile >= ntiles) return;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t tx = tile % tiles_x, ty = tile / tiles_x;
  const uint32_t x = tx * 8u + (lane & 7u), y = ty * 8u + (lane >> 3);
  const int64_t px = (int64_t)x * 256 + 128, py = (int64_t)y * 256 + 128;
  unsigned long long best = kRasterClear;
  if (toffs[ntiles] <= bin_cap) {
    const uint32_t b0 = toffs[tile], b1 = toffs[tile + 1];
    // the bin is fetched 64 entries at a time, one slot record per lane, then broadcast lane by lane
    for (uint32_t base = b0; base < b1; base += 64u) {
      const uint32_t cnt = min(64u, b1 - base);
      int32_t lx[3] = {0, 0, 0}, ly[3] = {0, 0, 0};
      float lz[3] = {0.0f, 0.0f, 0.0f};
      uint32_t lp = 0;
      if (lane < cnt) {
        const RasterSlot& q = slots[bins[base + lane]];
        for (int k = 0; k < 3; ++k) {
          lx[k] = q.x[k];
          ly[k] = q.y[k];
          lz[k] = q.z[k];
        }
        lp = q.prim;
      }
      raster_batch(cnt == 64u ? ~0ull : ((1ull << cnt) - 1ull), lx, ly, lz, lp, px, py, best);
    }
  } else {
    // the bins overflowed (more entries than the capacity sized from an earlier draw): the same
    // (slot, tile) pairs k_raster_bin would have binned, found by walking every slot
    for (uint32_t base = 0; base < nslots; base += 64u) {
      const uint32_t s = base + lane;
      int32_t lx[3] = {0, 0, 0}, ly[3] = {0, 0, 0};
      float lz[3] = {0.0f, 0.0f, 0.0f};
      uint32_t lp = 0;
      bool mine = false;
      if (s < nslots) {
        const uint32_t n = slot_tiles[s];
        if (n != 0) {
          const RasterSlot q = slots[s];
          const uint32_t dx = tx - q.tx0, dy = ty - q.ty0;  // unsigned: left / above the box wrap
          mine = dx < q.tw && (uint64_t)dy * q.tw + dx < n && tile_overlaps(q, tx, ty);
          for (int k = 0; k < 3; ++k) {
            lx[k] = q.x[k];
            ly[k] = q.y[k];
            lz[k] = q.z[k];
          }
          lp = q.prim;
        }
      }
      raster_batch(__builtin_amdgcn_ballot_w64(mine), lx, ly, lz, lp, px, py, best);
    }
  }
  if (x >= width || y >= height) return;
  const size_t o = (size_t)y * width + x;
  if (best == kRasterClear) {
    // ClearRenderTargetView {0.03, 0.35, 0.43, 1} (:529), depth 1.0 (:516)
    rgba8[o] = unorm8(0.03f) | (unorm8(0.35f) << 8) | (unorm8(0.43f) << 16) | (unorm8(1.0f) << 24);
    if (depth) depth[o] = 1.0f;
    return;
  }
  const uint32_t t = (uint32_t)(best & 0xffffffffu);
  uint32_t d = 0;
  while (d + 1 < drp->n && t >= drp->first[d + 1]) ++d;
  const uint32_t lt = t - drp->first[d];
  const float* vtx = drp->vtx[d];
  float col[3][4];
  for (int k = 0; k < 3; ++k) {
    const uint32_t vi = drp->idx[d] ? drp->idx[d][lt * 3 + k] : lt * 3 + k;
    const bool inside = vi + 1 < drp->nvtx[d];
    col[k][0] = inside ? vtx[vi * 6 + 3] : 0.0f;
    col[k][1] = inside ? vtx[vi * 6 + 4] : 0.0f;
    col[k][2] = inside ? vtx[vi * 6 + 5] : 0.0f;
    col[k][3] = inside ? vtx[(vi + 1) * 6 + 0] : 0.0f;
  }
  const float4 c0 = clip[(size_t)t * 3 + 0], c1 = clip[(size_t)t * 3 + 1], c2 = clip[(size_t)t * 3 + 2];
  // perspective-correct barycentrics of the pixel centre from the homogeneous (x, y, w) vertices
  const float qx = (((float)x + 0.5f) / (float)width) * 2.0f - 1.0f;
  const float qy = 1.0f - (((float)y + 0.5f) / (float)height) * 2.0f;
  const V3 h0 = v3(c0.x, c0.y, c0.w), h1 = v3(c1.x, c1.y, c1.w), h2 = v3(c2.x, c2.y, c2.w);
  const V3 q = v3(qx, qy, 1.0f);
  const float f0 = dot(cross(h1, h2), q), f1 = dot(cross(h2, h0), q), f2 = dot(cross(h0, h1), q);
  const float sum = (f0 + f1) + f2;
  const float w0 = f0 / sum, w1 = f1 / sum, w2 = f2 / sum;
  float out[4];
  for (int ch = 0; ch < 4; ++ch) out[ch] = (w0 * col[0][ch] + w1 * col[1][ch]) + w2 * col[2][ch];
  rgba8[o] = unorm8(out[0]) | (unorm8(out[1]) << 8) | (unorm8(out[2]) << 16) | (unorm8(out[3]) << 24);
  if (depth) depth[o] = __builtin_bit_cast(float, (uint32_t)(best >> 32));
}

}  // namespace

hipError_t launch_raster_bin(const RasterDraws& dr, const RasterView& rv, const RasterScratch& s,
                             hipStream_t stream) {
  const uint32_t nslots = dr.total * 7u;
  const uint32_t tx = (rv.width + 7) / 8, ty = (rv.height + 7) / 8, ntiles = tx * ty;
  hipError_t e = hipMemsetAsync(s.tcount, 0, (size_t)ntiles * 4, stream);
  if (e != hipSuccess) return e;
  if (dr.total) {
    k_raster_setup<<<(dr.total + kSetupBlock - 1) / kSetupBlock, kSetupBlock, 0, stream>>>(s.draws, dr.total, rv,
                                                                                          s.clip, s.slots, s.tiles);
    k_raster_bin<0><<<(nslots + 3) / 4, 256, 0, stream>>>(s.slots, s.tiles, nslots, tx, s.tcount, nullptr, nullptr, 0u);
  }
  const uint32_t nb = (ntiles + kScanBlock - 1) / kScanBlock;
  k_scan_blocks<<<nb, 1024, 0, stream>>>(s.tcount, ntiles, s.toffs, s.bsum);
  k_scan_sums<<<1, 1024, 0, stream>>>(s.bsum, nb, ntiles, s.toffs);
  if (nb > 1) k_scan_add<<<(ntiles + 255) / 256, 256, 0, stream>>>(s.toffs, ntiles, s.bsum);
  return hipGetLastError();
}

hipError_t launch_raster_draw(const RasterDraws& dr, const RasterView& rv, const RasterScratch& s, uint32_t bin_cap,
                              void* rgba8, float* depth, hipStream_t stream) {
  const uint32_t nslots = dr.total * 7u;
  const uint32_t tx = (rv.width + 7) / 8, ty = (rv.height + 7) / 8, ntiles = tx * ty;
  if (dr.total) {
    hipError_t e = hipMemsetAsync(s.tcount, 0, (size_t)ntiles * 4, stream);
    if (e != hipSuccess) return e;
    k_raster_bin<1><<<(nslots + 3) / 4, 256, 0, stream>>>(s.slots, s.tiles, nslots, tx, s.tcount, s.toffs, s.bins,
                                                          bin_cap);
  }
  k_raster_tile<<<(ntiles + 3) / 4, 256, 0, stream>>>(s.draws, s.clip, s.slots, s.toffs, s.bins, bin_cap, s.tiles,
                                                      nslots, tx, ntiles, rv.width, rv.height, (uint32_t*)rgba8, depth);
  return hipGetLastError();
}

}  // namespace rt
