// rt_lbvh.hip — on-device LBVH build for BLAS and TLAS on gfx950.
//
// Replaces the driver acceleration-structure builds behind
//   BottomLevelASGenerator::Generate  nv_helpers_dx12/BottomLevelASGenerator.cpp:177-245 (build :234)
//   TopLevelASGenerator::Generate     nv_helpers_dx12/TopLevelASGenerator.cpp:148-249 (build :239)
//
// Four schedules of the same tree (all deterministic, so oracle/rt_oracle.c rebuilds the bit-identical
// tree; build_path() picks one, RT_BUILD_PATH forces one for A/B):
//   2 <= n <= 512     k_build_tiny: one 512-thread workgroup, everything in LDS (rank sort, Apetrei
//                     climb, DP, expansion, BFS numbering), one launch
//   513 .. 8192       k_mid_*: rank sort, Apetrei climb with in-block LDS hand-offs, expansion, a
//                     one-workgroup top climb + BFS numbering, parallel node writes: four launches + one
//   n = 1             k_build_small: the multi-kernel stages in one 1024-thread workgroup
//   larger n          the multi-kernel pipeline:
//   1. centroid bounds      one 1024-thread workgroup, LDS min/max reduction (exact)
//   2. Morton codes         30-bit (10 bits/axis) of box centroids
//   3. LSD radix sort       4 passes x 8 bits; per pass: block digit histogram (LDS atomics),
//                           exclusive scan, stable scatter with wave64 ballot match + popcount
//                           ranks (keys tie-break on primitive index: stable)
//   4. Karras hierarchy     Karras 2012 over key64 = morton << 32 | leaf position
//   5. bottom-up refit      one thread per leaf, agent-scope release/acquire arrival counters,
//                           with the SAH collapse DP at each node
//   6. pack                 64-B child-pair nodes (both child boxes per node)
//   7. DP expansion + collapse into 4-wide BFS nodes, triangle gather into leaf order
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <vector>

#include "rt_internal.hpp"

#ifndef RT_FUSED_BUILD
#define RT_FUSED_BUILD 1  // n <= kFusedMax: the whole build in one workgroup (k_build_small)
#endif
#ifndef RT_FUSED_MAX_N
#define RT_FUSED_MAX_N 3072  // largest n built by k_build_small (measured crossover; capacity kFusedMax)
#endif
#ifndef RT_TINY_BUILD
#define RT_TINY_BUILD 1  // 2 <= n <= RT_TINY_MAX_N: the one-launch LDS build (k_build_tiny)
#endif
#ifndef RT_TINY_MAX_N
#define RT_TINY_MAX_N 512  // largest n built by k_build_tiny (capacity kTinyMax)
#endif
#ifndef RT_MID_BUILD
#define RT_MID_BUILD 1  // RT_MID_MIN_N <= n <= kMidMax: the five-launch build (k_mid_*)
#endif
#ifndef RT_MID_MIN_N
#define RT_MID_MIN_N 2  // smallest n built by k_mid_* (measured crossover against k_build_small)
#endif
#ifndef RT_REFIT_WT
#define RT_REFIT_WT 1  // multi-kernel refit: write-through hand-off instead of agent release/acquire fences
#endif
#ifndef RT_BUILD_TIMING
#define RT_BUILD_TIMING 0  // 1: k_build_small prints per-phase shader-clock counts (diagnostics)
#endif
#ifndef RT_SAH_COLLAPSE
#define RT_SAH_COLLAPSE 1  // SAH-optimal binary -> BVH4 collapse (DP); 0: greedy largest-area opening
#endif

namespace rt {
namespace {

constexpr int kRsThreads = 256;
constexpr int kRsRounds = 4;
constexpr int kRsTile = kRsThreads * kRsRounds;  // keys per workgroup per pass

__device__ __forceinline__ uint32_t expand_bits10(uint32_t x) {
  x = (x * 0x00010001u) & 0xFF0000FFu;
  x = (x * 0x00000101u) & 0x0F00F00Fu;
  x = (x * 0x00000011u) & 0xC30C30C3u;
  x = (x * 0x00000005u) & 0x49249249u;
  return x;
}

__device__ __forceinline__ uint32_t quantize10(float c, float lo, float inv_ext) {
  float q = (c - lo) * inv_ext;
  float s = q * 1024.0f;
  s = fminf(fmaxf(s, 0.0f), 1023.0f);
  return (uint32_t)s;
}

// 1. centroid bounds + union of prim boxes. out[0..5] centroid lo/hi, out[6..11] box lo/hi.
__global__ __launch_bounds__(1024) void k_bounds(const float* __restrict__ box, uint32_t n,
                                                 float* __restrict__ out) {
  __shared__ float red[12][1024 / 64];
  float v[12];
  for (int k = 0; k < 3; ++k) {
    v[k] = INFINITY;
    v[3 + k] = -INFINITY;
    v[6 + k] = INFINITY;
    v[9 + k] = -INFINITY;
  }
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    const float* b = box + (size_t)i * 6;
    for (int k = 0; k < 3; ++k) {
      float c = (b[k] + b[3 + k]) * 0.5f;
      v[k] = fminf(v[k], c);
      v[3 + k] = fmaxf(v[3 + k], c);
      v[6 + k] = fminf(v[6 + k], b[k]);
      v[9 + k] = fmaxf(v[9 + k], b[3 + k]);
    }
  }
  // wave64 reduction, then across the 16 waves
  for (int off = 32; off >= 1; off >>= 1) {
    for (int k = 0; k < 12; ++k) {
      float o = __shfl_xor(v[k], off, 64);
      bool is_min = (k % 6) < 3;
      v[k] = is_min ? fminf(v[k], o) : fmaxf(v[k], o);
    }
  }
  int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0)
    for (int k = 0; k < 12; ++k) red[k][w] = v[k];
  __syncthreads();
  if (threadIdx.x < 12) {
    int k = threadIdx.x;
    bool is_min = (k % 6) < 3;
    float r = red[k][0];
    for (int j = 1; j < (int)(blockDim.x / 64); ++j) r = is_min ? fminf(r, red[k][j]) : fmaxf(r, red[k][j]);
    out[k] = r;
  }
}

// 2. Morton codes of box centroids; values = primitive index.
__global__ void k_morton(const float* __restrict__ box, uint32_t n, const float* __restrict__ cb,
                         uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* b = box + (size_t)i * 6;
  uint32_t q[3];
  for (int k = 0; k < 3; ++k) {
    float ext = cb[3 + k] - cb[k];
    float inv = ext > 0.0f ? 1.0f / ext : 0.0f;
    float c = (b[k] + b[3 + k]) * 0.5f;
    q[k] = quantize10(c, cb[k], inv);
  }
  keys[i] = (expand_bits10(q[0]) << 2) | (expand_bits10(q[1]) << 1) | expand_bits10(q[2]);
  vals[i] = i;
}

// 3a. per-workgroup digit histogram, stored digit-major: hist[d * nblocks + b].
__global__ __launch_bounds__(kRsThreads) void k_rs_hist(const uint32_t* __restrict__ keys, uint32_t n,
                                                         int shift, uint32_t* __restrict__ hist,
                                                         uint32_t nblocks) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  uint32_t base = blockIdx.x * kRsTile;
  for (int r = 0; r < kRsRounds; ++r) {
    uint32_t i = base + r * kRsThreads + threadIdx.x;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & 255u], 1u);
  }
  __syncthreads();
  hist[threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];
}

// 3b. exclusive scan of len values in place, one 1024-thread workgroup.
__global__ __launch_bounds__(1024) void k_rs_scan(uint32_t* __restrict__ data, uint32_t len) {
  __shared__ uint32_t sums[1024];
  uint32_t per = (len + 1023u) / 1024u;
  uint32_t b = threadIdx.x * per, e = min(b + per, len);
  uint32_t s = 0;
  for (uint32_t i = b; i < e; ++i) s += data[i];
  sums[threadIdx.x] = s;
  __syncthreads();
  for (uint32_t off = 1; off < 1024; off <<= 1) {
    uint32_t add = threadIdx.x >= off ? sums[threadIdx.x - off] : 0u;
    __syncthreads();
    sums[threadIdx.x] += add;
    __syncthreads();
  }
  uint32_t run = sums[threadIdx.x] - s;  // exclusive
  for (uint32_t i = b; i < e; ++i) {
    uint32_t v = data[i];
    data[i] = run;
    run += v;
  }
}

// 3c. stable scatter. Each round a wave ranks its 64 keys by digit with 8 ballots (peer mask of
// equal digits) + popcount of lower peers; waves of a workgroup are ordered through LDS counts.
__global__ __launch_bounds__(kRsThreads) void k_rs_scatter(const uint32_t* __restrict__ kin,
                                                            const uint32_t* __restrict__ vin,
                                                            uint32_t* __restrict__ kout,
                                                            uint32_t* __restrict__ vout, uint32_t n,
                                                            int shift, const uint32_t* __restrict__ scan,
                                                            uint32_t nblocks) {
  __shared__ uint32_t offs[256];
  __shared__ uint32_t wcnt[kRsThreads / 64][256];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
  offs[tid] = scan[tid * nblocks + blockIdx.x];
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64u - lane));
  const uint32_t base = blockIdx.x * kRsTile;
  for (int r = 0; r < kRsRounds; ++r) {
    for (int k = 0; k < kRsThreads / 64; ++k) wcnt[k][tid] = 0;
    __syncthreads();
    uint32_t i = base + r * kRsThreads + tid;
    bool valid = i < n;
    uint32_t key = valid ? kin[i] : 0u;
    uint32_t val = valid ? vin[i] : 0u;
    uint32_t digit = (key >> shift) & 255u;
    uint64_t peers = __ballot(valid);
    for (int b = 0; b < 8; ++b) {
      bool bit = (digit >> b) & 1u;
      uint64_t m = __ballot(valid && bit);
      peers &= bit ? m : ~m;
    }
    uint32_t rank = (uint32_t)__popcll(peers & lt);
    if (valid && rank == 0) wcnt[w][digit] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (valid) {
      uint32_t pre = 0;
      for (uint32_t k = 0; k < w; ++k) pre += wcnt[k][digit];
      uint32_t pos = offs[digit] + pre + rank;
      kout[pos] = key;
      vout[pos] = val;
    }
    __syncthreads();
    uint32_t tot = 0;
    for (int k = 0; k < kRsThreads / 64; ++k) tot += wcnt[k][tid];
    offs[tid] += tot;
    __syncthreads();
  }
}

__device__ __forceinline__ int delta(const uint32_t* __restrict__ keys, int n, int i, int j) {
  if (j < 0 || j >= n) return -1;
  uint64_t a = ((uint64_t)keys[i] << 32) | (uint32_t)i;
  uint64_t b = ((uint64_t)keys[j] << 32) | (uint32_t)j;
  return __clzll(a ^ b);
}

// 4. Karras 2012 hierarchy: internal node i, children encoded >= 0 internal / ~leaf.
__global__ void k_karras(const uint32_t* __restrict__ keys, int n, int* __restrict__ child,
                         int* __restrict__ parent_int, int* __restrict__ parent_leaf) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n - 1) return;
  int d = (delta(keys, n, i, i + 1) - delta(keys, n, i, i - 1)) >= 0 ? 1 : -1;
  int dmin = delta(keys, n, i, i - d);
  int lmax = 2;
  while (delta(keys, n, i, i + lmax * d) > dmin) lmax <<= 1;
  int l = 0;
  for (int t = lmax >> 1; t >= 1; t >>= 1)
    if (delta(keys, n, i, i + (l + t) * d) > dmin) l += t;
  int j = i + l * d;
  int dnode = delta(keys, n, i, j);
  int s = 0, t = l;
  while (true) {
    t = (t + 1) >> 1;
    if (delta(keys, n, i, i + (s + t) * d) > dnode) s += t;
    if (t <= 1) break;
  }
  int gamma = i + s * d + (d < 0 ? d : 0);
  int lo = i < j ? i : j, hi = i < j ? j : i;
  int left = (lo == gamma) ? ~gamma : gamma;
  int right = (hi == gamma + 1) ? ~(gamma + 1) : gamma + 1;
  child[2 * i] = left;
  child[2 * i + 1] = right;
  if (left >= 0) parent_int[left] = i; else parent_leaf[~left] = i;
  if (right >= 0) parent_int[right] = i; else parent_leaf[~right] = i;
  if (i == 0) parent_int[0] = -1;
}

__device__ __forceinline__ void load_box(int c, const float* __restrict__ nbox,
                                         const float* __restrict__ primbox,
                                         const uint32_t* __restrict__ sorted, float b[6]) {
  const float* p = c >= 0 ? nbox + (size_t)c * 6 : primbox + (size_t)sorted[~c] * 6;
  for (int k = 0; k < 6; ++k) b[k] = p[k];
}

// 5. bottom-up refit. The second arrival at a node computes its box. Hand-off follows the
// agent-scope release -> counter -> acquire protocol (node boxes may be cached on other XCDs).
__device__ __forceinline__ float half_area6(const float* b) {
  const float dx = b[3] - b[0], dy = b[4] - b[1], dz = b[5] - b[2];
  return (dx * dy + dy * dz) + dz * dx;
}

// SAH-optimal collapse DP at binary node `node` with box bb and children c0, c1 (>= 0: internal,
// DP already final; < 0: a triangle / instance leaf, cost 0). The cost of a collapse is the sum of
// its wide nodes' half areas: a wide node's visit tests all four slots, and every triangle is tested
// under the same conditions whatever the collapse. C(n, i) = least cost of n's subtree as at most i
// slot roots: D(n, i) = min_j C(c0, j) + C(c1, i - j), C(n, 1) = A(n) + D(n, 4) (n is a wide node),
// C(n, i) = min(C(n, 1), D(n, i)). dpc[n] = C(n, 1..4); dps[n] byte i-1 = 0 when n is a wide node
// for i slots, else j (the slots of c0). Strict < keeps the lowest j; oracle dp_prepare is the same
// arithmetic in the same order.
__device__ __forceinline__ void sah_dp_vals(const float* bb, float4 l, float4 r, float4& out_c, uint32_t& out_s) {
  const float cl[5] = {0.0f, l.x, l.y, l.z, l.w}, cr[5] = {0.0f, r.x, r.y, r.z, r.w};
  float D[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
  uint32_t J[5] = {0, 0, 0, 0, 0};
  for (int i = 2; i <= 4; ++i) {
    D[i] = INFINITY;
    J[i] = 1;
    for (int j = 1; j < i; ++j) {
      const float c = cl[j] + cr[i - j];
      if (c < D[i]) {
        D[i] = c;
        J[i] = (uint32_t)j;
      }
    }
  }
  const float self = half_area6(bb) + D[4];
  float C[5];
  uint32_t S = 0;
  C[1] = self;
  for (int i = 2; i <= 4; ++i) {
    const bool split = D[i] < self;
    C[i] = split ? D[i] : self;
    S |= (split ? J[i] : 0u) << (8 * (i - 1));
  }
  out_c = make_float4(C[1], C[2], C[3], C[4]);
  out_s = S;
}

__device__ __forceinline__ void sah_dp(int node, const float* bb, int c0, int c1, float4* __restrict__ dpc,
                                       uint32_t* __restrict__ dps) {
  const float4 zero = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  const float4 l = c0 >= 0 ? dpc[c0] : zero, r = c1 >= 0 ? dpc[c1] : zero;
  float4 c;
  uint32_t sj;
  sah_dp_vals(bb, l, r, c, sj);
  dpc[node] = c;
  dps[node] = sj;
}

// Write-through hand-off (MI355X_MICROARCH.md, handoff-flag: sc1 payload -> vmcnt(0) -> flag):
// agent-scope relaxed stores / loads are the sc1 forms, coherent across the XCDs' L2s without the
// L2 write-back an agent-scope release fence issues at every level of the climb.
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_refit(int n, const int* __restrict__ parent_leaf, const int* __restrict__ parent_int,
                        const int* __restrict__ child, const float* __restrict__ primbox,
                        const uint32_t* __restrict__ sorted, float* nbox, uint32_t* flags,
                        float4* __restrict__ dpc, uint32_t* __restrict__ dps) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int node = parent_leaf[i];
#if RT_REFIT_WT
  // the node records of the climb (box, DP costs, DP choices) move by write-through stores and
  // coherent loads; a climbing thread's stores are complete (vmcnt(0)) before its arrival counts
  while (node >= 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(&flags[node], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == 0) return;
    const int c[2] = {child[2 * node], child[2 * node + 1]};
    float cb[2][6];
    float4 cd[2];
    for (int k = 0; k < 2; ++k) {
      cd[k] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      if (c[k] >= 0) {
        const float* p = nbox + (size_t)c[k] * 6;
        for (int q = 0; q < 6; ++q) cb[k][q] = ld_wt(p + q);
        if (dpc) {
          const float* d = (const float*)(dpc + c[k]);
          cd[k] = make_float4(ld_wt(d), ld_wt(d + 1), ld_wt(d + 2), ld_wt(d + 3));
        }
      } else {
        const float* p = primbox + (size_t)sorted[~c[k]] * 6;
        for (int q = 0; q < 6; ++q) cb[k][q] = p[q];
      }
    }
    float bb[6];
    for (int k = 0; k < 3; ++k) {
      bb[k] = fminf(cb[0][k], cb[1][k]);
      bb[3 + k] = fmaxf(cb[0][3 + k], cb[1][3 + k]);
    }
    float* o = nbox + (size_t)node * 6;
    for (int k = 0; k < 6; ++k) st_wt(o + k, bb[k]);
    if (dpc) {
      float4 dc;
      uint32_t sj;
      sah_dp_vals(bb, cd[0], cd[1], dc, sj);
      float* d = (float*)(dpc + node);
      st_wt(d, dc.x);
      st_wt(d + 1, dc.y);
      st_wt(d + 2, dc.z);
      st_wt(d + 3, dc.w);
      dps[node] = sj;  // read only by later kernels
    }
    node = parent_int[node];
  }
#else
  while (node >= 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t old = __hip_atomic_fetch_add(&flags[node], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == 0) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    float a[6], b[6];
    load_box(child[2 * node], nbox, primbox, sorted, a);
    load_box(child[2 * node + 1], nbox, primbox, sorted, b);
    float* o = nbox + (size_t)node * 6;
    float bb[6];
    for (int k = 0; k < 3; ++k) {
      bb[k] = fminf(a[k], b[k]);
      bb[3 + k] = fmaxf(a[3 + k], b[3 + k]);
    }
    for (int k = 0; k < 6; ++k) o[k] = bb[k];
    if (dpc) sah_dp(node, bb, child[2 * node], child[2 * node + 1], dpc, dps);
    node = parent_int[node];
  }
#endif
}

// 6. pack child-pair nodes.
__global__ void k_pack(int n, const int* __restrict__ child, const float* __restrict__ nbox,
                       const float* __restrict__ primbox, const uint32_t* __restrict__ sorted,
                       bool leaf_ref_is_prim, BinNode* __restrict__ nodes) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n - 1) return;
  BinNode nd;
  int c[2] = {child[2 * i], child[2 * i + 1]};
  float b[2][6];
  for (int k = 0; k < 2; ++k) load_box(c[k], nbox, primbox, sorted, b[k]);
  for (int k = 0; k < 3; ++k) {
    nd.lo0[k] = b[0][k];
    nd.hi0[k] = b[0][3 + k];
    nd.lo1[k] = b[1][k];
    nd.hi1[k] = b[1][3 + k];
  }
  for (int k = 0; k < 2; ++k)
    if (c[k] < 0 && leaf_ref_is_prim) c[k] = ~(int)sorted[~c[k]];
  nd.c0 = c[0];
  nd.c1 = c[1];
  nd.pad0 = nd.pad1 = 0;
  nodes[i] = nd;
}

// n == 1: a root whose two children are the single leaf (tested twice; ties keep the result).
__global__ void k_single(const float* __restrict__ primbox, bool leaf_ref_is_prim, BinNode* nodes) {
  BinNode nd;
  for (int k = 0; k < 3; ++k) {
    nd.lo0[k] = nd.lo1[k] = primbox[k];
    nd.hi0[k] = nd.hi1[k] = primbox[3 + k];
  }
  nd.c0 = ~0;  // ~slot 0 == ~prim 0
  nd.c1 = kEmptyChild;
  (void)leaf_ref_is_prim;
  nd.pad0 = nd.pad1 = 0;
  nodes[0] = nd;
}

// 7. collapse the binary tree into 4-wide nodes in BFS order (children chosen by gather4_dp from
// the SAH DP of k_refit; gather4, the greedy largest-area opening, with RT_SAH_COLLAPSE=0). One
// workgroup walks the levels; each level's new node indices come from a block-wide exclusive
// scan of per-node internal-child counts (deterministic, no atomics), so the oracle's sequential
// BFS yields the same array. Unused slots get kEmptyChild and the box lo = hi = +inf, which
// every slab test rejects (min/max and near/far forms alike: t is +inf or -inf on every axis),
// so traversal needs no per-slot validity mask.
// It also bounds the traversal stack: a visited node pushes (count - 1) siblings, so the most a
// root-to-node path can leave on the stack is ps[node] + count(node) - 1, ps = sum over the
// ancestors. info[0] = node count, info[1] = levels, info[2] = that maximum.
// Half surface area of a box (the SAH weight), summed in a fixed order (mirrored by the oracle).
__device__ __forceinline__ float half_area(const float* b) {
  const float dx = b[3] - b[0], dy = b[4] - b[1], dz = b[5] - b[2];
  return (dx * dy + dy * dz) + dz * dx;
}

// Children of one 4-wide node rooted at binary node `root`: start from its two children and
// open the internal candidate with the largest surface area (lowest slot on ties) until there
// are four, so the wide nodes come out full and the large boxes are split first.
__device__ __forceinline__ int gather4(const BinNode* __restrict__ bin, int root, int ref[4], float box[4][6]) {
  const BinNode& b = bin[root];
  ref[0] = b.c0;
  ref[1] = b.c1;
  for (int a = 0; a < 3; ++a) {
    box[0][a] = b.lo0[a];
    box[0][3 + a] = b.hi0[a];
    box[1][a] = b.lo1[a];
    box[1][3 + a] = b.hi1[a];
  }
  int cnt = 2;
  while (cnt < 4) {
    int best = -1;
    float bsa = 0.0f;
    for (int j = 0; j < cnt; ++j) {
      if (ref[j] < 0) continue;
      const float sa = half_area(box[j]);
      if (best < 0 || sa > bsa) {
        best = j;
        bsa = sa;
      }
    }
    if (best < 0) break;
    const BinNode& g = bin[ref[best]];
    ref[best] = g.c0;
    ref[cnt] = g.c1;
    for (int a = 0; a < 3; ++a) {
      box[best][a] = g.lo0[a];
      box[best][3 + a] = g.hi0[a];
      box[cnt][a] = g.lo1[a];
      box[cnt][3 + a] = g.hi1[a];
    }
    ++cnt;
  }
  return cnt;
}

// Children of the 4-wide node rooted at binary node `root` under the collapse DP: the root's four
// slots split between its children as D(root, 4) chose, each child expanded while its choice for
// its slot count is a split (left first; mirrors oracle gather4_dp / dp_expand).
__device__ __forceinline__ int gather4_dp(const BinNode* __restrict__ bin, const float4* __restrict__ dpc,
                                          const uint32_t* __restrict__ dps, int root, int ref[4], float box[4][6]) {
  const BinNode& b = bin[root];
  const float4 zero = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  const float4 l = b.c0 >= 0 ? dpc[b.c0] : zero, r = b.c1 >= 0 ? dpc[b.c1] : zero;
  const float cl[4] = {l.x, l.y, l.z, l.w}, cr[4] = {r.x, r.y, r.z, r.w};
  int bj = 1;
  float bc = INFINITY;
  for (int j = 1; j < 4; ++j) {
    const float c = cl[j - 1] + cr[4 - j - 1];
    if (c < bc) {
      bc = c;
      bj = j;
    }
  }
  // explicit stack of (ref, slots, box); right pushed before left so slots come out left first
  int sref[4], sk[4];
  float sbox[4][6];
  int top = 0;
  sref[top] = b.c1;
  sk[top] = 4 - bj;
  for (int a = 0; a < 3; ++a) {
    sbox[top][a] = b.lo1[a];
    sbox[top][3 + a] = b.hi1[a];
  }
  ++top;
  sref[top] = b.c0;
  sk[top] = bj;
  for (int a = 0; a < 3; ++a) {
    sbox[top][a] = b.lo0[a];
    sbox[top][3 + a] = b.hi0[a];
  }
  ++top;
  int cnt = 0;
  while (top > 0) {
    --top;
    const int c = sref[top], k = sk[top];
    const uint32_t j = c >= 0 ? (dps[c] >> (8 * (k - 1))) & 0xffu : 0u;
    if (j == 0) {
      ref[cnt] = c;
      for (int a = 0; a < 6; ++a) box[cnt][a] = sbox[top][a];
      ++cnt;
      continue;
    }
    const BinNode& g = bin[c];
    sref[top] = g.c1;
    sk[top] = k - (int)j;
    for (int a = 0; a < 3; ++a) {
      sbox[top][a] = g.lo1[a];
      sbox[top][3 + a] = g.hi1[a];
    }
    ++top;
    sref[top] = g.c0;
    sk[top] = (int)j;
    for (int a = 0; a < 3; ++a) {
      sbox[top][a] = g.lo0[a];
      sbox[top][3 + a] = g.hi0[a];
    }
    ++top;
  }
  return cnt;
}

// BLAS nodes keep their internal children in the lowest slots (stable: ascending half area within
// the internal and within the leaf children). The walk tests a node's entered triangles in place and
// then orders only its internal children, so this changes no visit order and no counter; with it, an
// internal child's ref is first_inner + slot (the packet stack pops without a popcount).
template <int M>
__device__ __forceinline__ void inner_first(int (&ref)[M], float (&box)[M][6]) {
#pragma unroll
  for (int x = 1; x < M; ++x)
#pragma unroll
    for (int y = x; y > 0; --y)
      if (ref[y] >= 0 && ref[y - 1] < 0) {
        const int tr = ref[y];
        ref[y] = ref[y - 1];
        ref[y - 1] = tr;
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          const float t = box[y][q];
          box[y][q] = box[y - 1][q];
          box[y - 1][q] = t;
        }
      }
}

// The DP expansion of every binary node, in parallel (only wide-node roots are read): k_collapse
// then takes one record per node instead of walking dependent loads level by level.
struct alignas(128) Exp4 {
  int ref[4];
  float box[4][6];
  int cnt, pad[3];
};

__global__ void k_dp_expand(int nbin, const BinNode* __restrict__ bin, const float4* __restrict__ dpc,
                            const uint32_t* __restrict__ dps, Exp4* __restrict__ exp, bool blas) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nbin) return;
  Exp4 e;
  e.cnt = gather4_dp(bin, dpc, dps, i, e.ref, e.box);
  // slots by ascending half area (stable): nearest-first ties (rays starting inside several child
  // boxes) and the any-hit lowest-slot order then visit the tighter box first
  for (int a = 1; a < e.cnt; ++a)
    for (int b = a; b > 0 && half_area6(e.box[b]) < half_area6(e.box[b - 1]); --b) {
      const int tr = e.ref[b];
      e.ref[b] = e.ref[b - 1];
      e.ref[b - 1] = tr;
      for (int q = 0; q < 6; ++q) {
        const float t = e.box[b][q];
        e.box[b][q] = e.box[b - 1][q];
        e.box[b - 1][q] = t;
      }
    }
  for (int j = e.cnt; j < 4; ++j) e.ref[j] = kEmptyChild;
  if (blas) inner_first(e.ref, e.box);
  e.pad[0] = e.pad[1] = e.pad[2] = 0;
  exp[i] = e;
}

constexpr int kFusedThreads = 1024;
constexpr int kFusedWaves = kFusedThreads / 64;
constexpr uint32_t kFusedMax = 8192;  // keys + values, double-buffered in LDS: 128 KiB
static_assert(RT_FUSED_MAX_N <= kFusedMax, "the one-workgroup build holds at most kFusedMax keys");

// Exclusive prefix sum of one value per thread over the workgroup, in thread order; *total gets
// the sum. Two barriers (a wave scan by shuffles, then the 16 wave totals through LDS).
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_w, uint32_t* total) {
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off, 64);
    x += lane >= (uint32_t)off ? y : 0u;
  }
  if (lane == 63u) s_w[w] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < kFusedWaves; ++k) {
    const uint32_t c = s_w[k];
    pre += (uint32_t)k < w ? c : 0u;
    tot += c;
  }
  __syncthreads();  // s_w is reused by the next call
  *total = tot;
  return pre + x - v;
}

__global__ __launch_bounds__(1024) void k_collapse(const BinNode* __restrict__ bin, const Exp4* __restrict__ exp,
                                                   Bvh4Node* __restrict__ out,
                                                   int* la, int* lb, int* ps, uint32_t* __restrict__ info,
                                                   bool blas) {
  __shared__ uint32_t s_w[kFusedWaves];
  __shared__ int s_maxstack;
  const int tid = threadIdx.x;
  int* cur = la;
  int* nxt = lb;
  if (tid == 0) {
    cur[0] = 0;
    ps[0] = 0;
    s_maxstack = 0;
  }
  __syncthreads();
  int lmax = 0;
  int cur_n = 1, base = 0, depth = 0;
  while (cur_n > 0) {
    ++depth;
    int next_total = 0;
    for (int cs = 0; cs < cur_n; cs += 1024) {
      const int i = cs + tid;
      const bool valid = i < cur_n;
      int ref[4];
      float box[4][6];
      int cnt = 0;
      if (valid) {
        if (exp) {
          const Exp4& e = exp[cur[i]];
          cnt = e.cnt;
          for (int j = 0; j < 4; ++j) {
            ref[j] = e.ref[j];
            for (int a = 0; a < 6; ++a) box[j][a] = e.box[j][a];
          }
        } else {
          cnt = gather4(bin, cur[i], ref, box);
          for (int j = cnt; j < 4; ++j) ref[j] = kEmptyChild;
          if (blas) inner_first(ref, box);
        }
      }
      uint32_t m = 0;
      for (int j = 0; j < cnt; ++j) m += ref[j] >= 0;
      uint32_t tot;
      const int excl = (int)block_excl_scan(m, s_w, &tot);
      const int chunk_total = (int)tot;
      if (valid) {
        Bvh4Node nd;
        int o = excl;
        const int below = ps[base + i] + cnt - 1;
        lmax = below > lmax ? below : lmax;
        uint32_t valid = 0, inner = 0;
        nd.first_inner = 0;
        for (int j = 0; j < 4; ++j) {
          const float inf = __builtin_inff();
          float b6[6] = {inf, inf, inf, inf, inf, inf};
          int32_t r = kEmptyChild;
          if (j < cnt && ref[j] != kEmptyChild) {
            ++valid;
            for (int a = 0; a < 6; ++a) b6[a] = box[j][a];
            if (ref[j] >= 0) {
              const int pos = next_total + o;
              nxt[pos] = ref[j];
              r = base + cur_n + pos;
              ps[r] = below;
              if (o == excl) nd.first_inner = r;
              inner |= 1u << j;
              ++o;
            } else {
              r = ref[j];
            }
          }
          nd.lox[j] = b6[0];
          nd.loy[j] = b6[1];
          nd.loz[j] = b6[2];
          nd.hix[j] = b6[3];
          nd.hiy[j] = b6[4];
          nd.hiz[j] = b6[5];
          nd.child[j] = r;
        }
        nd.count = valid;
        nd.inner_mask = inner;
        nd.entry_base = ((uint32_t)nd.first_inner << 8) | (inner << 4);
        out[base + i] = nd;
      }
      next_total += chunk_total;
      __syncthreads();
    }
    int* t = cur;
    cur = nxt;
    nxt = t;
    base += cur_n;
    cur_n = next_total;
  }
  atomicMax(&s_maxstack, lmax);
  __syncthreads();
  if (tid == 0) {
    info[0] = (uint32_t)base;
    info[1] = (uint32_t)depth;
    info[2] = (uint32_t)s_maxstack;
  }
}

// ------------------------------------------------------------------------------------------
// Fused small-N build: every stage above in ONE 1024-thread workgroup (n <= kFusedMax), the
// per-stage launches and the device-scope hand-offs replaced by workgroup barriers and LDS.
// Same arithmetic in the same order as the multi-kernel path, so the tree is bitwise the same:
//   bounds      the k_bounds reduction (exact min / max)
//   morton      keys and values straight into LDS
//   radix sort  4 x 8-bit LSD passes LDS -> LDS; each wave owns a contiguous chunk, ranks its
//               64 keys per round with 8 ballots; one block scan of the (digit, wave) counts per
//               pass orders digits, then waves, then rounds, then lanes: stable, like k_rs_*
//   Karras      from the sorted keys in LDS
//   refit + DP  the leaf-to-root climb with the arrival counters in LDS (workgroup-scope
//               atomics: no L2 write-back per level as the agent-scope hand-off of k_refit needs)
//   pack, DP expansion, collapse (level lists and stack sums in LDS, wave-scan prefix sums)
//   + the triangle gather into leaf order (BLAS).
// Teapot (6320 triangles): ~20 launches -> 1.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int delta_lds(const uint32_t* keys, int n, int i, int j) {
  if (j < 0 || j >= n) return -1;
  const uint64_t a = ((uint64_t)keys[i] << 32) | (uint32_t)i;
  const uint64_t b = ((uint64_t)keys[j] << 32) | (uint32_t)j;
  return __clzll(a ^ b);
}

// gather4_dp without a local stack (registers only: the one-workgroup build cannot hide scratch
// latency). A slot is (ref, parent binary node, side); its box is read from the parent afterwards.
// The expansion is the same recursion in the same left-to-right order: the DP hands a child k of
// the root's four slots, and a child given k > 1 slots is split as dps chose (0: kept whole).
struct Slots4 {
  int ref[4], par[4], side[4];
  int cnt;
};
__device__ __forceinline__ void put_slot(Slots4& s, int ref, int par, int side) {
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (s.cnt == q) {
      s.ref[q] = ref;
      s.par[q] = par;
      s.side[q] = side;
    }
  ++s.cnt;
}
template <int K>
__device__ __forceinline__ void expand_slots(const BinNode* __restrict__ bin, const uint32_t* __restrict__ dps, int c,
                                             int par, int side, Slots4& s) {
  if (K == 1 || c < 0) {
    put_slot(s, c, par, side);
    return;
  }
  const uint32_t j = (dps[c] >> (8 * (K - 1))) & 0xffu;
  if (j == 0) {
    put_slot(s, c, par, side);
    return;
  }
  const int2 g = *reinterpret_cast<const int2*>(&bin[c].c0);
  if (K == 2) {
    expand_slots<1>(bin, dps, g.x, c, 0, s);
    expand_slots<1>(bin, dps, g.y, c, 1, s);
  } else if (j == 1) {
    expand_slots<1>(bin, dps, g.x, c, 0, s);
    expand_slots<(K > 2 ? K - 1 : 1)>(bin, dps, g.y, c, 1, s);
  } else {
    expand_slots<(K > 2 ? K - 1 : 1)>(bin, dps, g.x, c, 0, s);
    expand_slots<1>(bin, dps, g.y, c, 1, s);
  }
}

// The wide node rooted at binary node `root` (gather4_dp + the k_dp_expand slot order), in registers.
__device__ __forceinline__ int wide_slots_dp(const BinNode* __restrict__ bin, const float4* __restrict__ dpc,
                                             const uint32_t* __restrict__ dps, int root, int (&ref)[4],
                                             float (&box)[4][6], bool blas) {
  const int2 rc = *reinterpret_cast<const int2*>(&bin[root].c0);
  const float4 zero = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  const float4 l = rc.x >= 0 ? dpc[rc.x] : zero, r = rc.y >= 0 ? dpc[rc.y] : zero;
  const float cl[4] = {l.x, l.y, l.z, l.w}, cr[4] = {r.x, r.y, r.z, r.w};
  int bj = 1;
  float bc = INFINITY;
#pragma unroll
  for (int j = 1; j < 4; ++j) {
    const float c = cl[j - 1] + cr[4 - j - 1];
    if (c < bc) {
      bc = c;
      bj = j;
    }
  }
  Slots4 s;
  s.cnt = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) s.ref[q] = s.par[q] = s.side[q] = 0;
  if (bj == 1) {
    expand_slots<1>(bin, dps, rc.x, root, 0, s);
    expand_slots<3>(bin, dps, rc.y, root, 1, s);
  } else if (bj == 2) {
    expand_slots<2>(bin, dps, rc.x, root, 0, s);
    expand_slots<2>(bin, dps, rc.y, root, 1, s);
  } else {
    expand_slots<3>(bin, dps, rc.x, root, 0, s);
    expand_slots<1>(bin, dps, rc.y, root, 1, s);
  }
  float a[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    ref[q] = s.ref[q];
    const BinNode& pb = bin[s.par[q]];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      box[q][k] = q < s.cnt ? (s.side[q] ? pb.lo1[k] : pb.lo0[k]) : 0.0f;
      box[q][3 + k] = q < s.cnt ? (s.side[q] ? pb.hi1[k] : pb.hi0[k]) : 0.0f;
    }
    a[q] = half_area6(box[q]);
  }
  // ascending half area, stable (k_dp_expand's insertion sort with every comparison unrolled: once
  // an element stops, the comparisons below it find the prefix sorted and swap nothing)
#pragma unroll
  for (int x = 1; x < 4; ++x)
#pragma unroll
    for (int y = x; y > 0; --y)
      if (x < s.cnt && a[y] < a[y - 1]) {
        const float ta = a[y];
        a[y] = a[y - 1];
        a[y - 1] = ta;
        const int tr = ref[y];
        ref[y] = ref[y - 1];
        ref[y - 1] = tr;
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          const float t = box[y][q];
          box[y][q] = box[y - 1][q];
          box[y - 1][q] = t;
        }
      }
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (j >= s.cnt) ref[j] = kEmptyChild;
  if (blas) inner_first(ref, box);
  return s.cnt;
}

__global__ __launch_bounds__(kFusedThreads) void k_build_small(
    const float* __restrict__ primbox, uint32_t n, bool leaf_ref_is_prim, uint32_t* __restrict__ sorted,
    float* __restrict__ cb_out, int* __restrict__ pleaf, float* nbox, float4* dpc, uint32_t* dps, BinNode* bin,
    Bvh4Node* __restrict__ out,
    uint32_t* __restrict__ info, const TriRec* __restrict__ tri_in, TriRec* __restrict__ tri_out) {
  // LDS: sort buffers (keys A | values A | keys B | values B) + (digit, wave) counts; later
  // phases reuse the same words: arrival flags (refit), level lists and stack sums (collapse)
  __shared__ uint32_t s_mem[4 * kFusedMax + 256 * kFusedWaves];
  __shared__ float s_red[12][kFusedWaves];
  __shared__ float s_cb[12];
  __shared__ uint32_t s_w[kFusedWaves];
  __shared__ int s_maxstack;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
#if RT_BUILD_TIMING
  uint64_t bt[9];
  bt[0] = __builtin_amdgcn_s_memtime();
#define RT_BT(k) bt[k] = __builtin_amdgcn_s_memtime()
#else
#define RT_BT(k) (void)0
#endif
  uint32_t* keyA = s_mem;
  uint32_t* valA = s_mem + kFusedMax;
  uint32_t* keyB = s_mem + 2 * kFusedMax;
  uint32_t* valB = s_mem + 3 * kFusedMax;
  uint32_t* cnt = s_mem + 4 * kFusedMax;  // [wave][digit]: a wave's lanes hit distinct banks

  // 1. bounds (k_bounds)
  {
    float v[12];
    for (int k = 0; k < 3; ++k) {
      v[k] = INFINITY;
      v[3 + k] = -INFINITY;
      v[6 + k] = INFINITY;
      v[9 + k] = -INFINITY;
    }
    for (uint32_t i = tid; i < n; i += kFusedThreads) {
      const float* b = primbox + (size_t)i * 6;
      for (int k = 0; k < 3; ++k) {
        const float c = (b[k] + b[3 + k]) * 0.5f;
        v[k] = fminf(v[k], c);
        v[3 + k] = fmaxf(v[3 + k], c);
        v[6 + k] = fminf(v[6 + k], b[k]);
        v[9 + k] = fmaxf(v[9 + k], b[3 + k]);
      }
    }
    for (int off = 32; off >= 1; off >>= 1)
      for (int k = 0; k < 12; ++k) {
        const float o = __shfl_xor(v[k], off, 64);
        v[k] = (k % 6) < 3 ? fminf(v[k], o) : fmaxf(v[k], o);
      }
    if (lane == 0)
      for (int k = 0; k < 12; ++k) s_red[k][w] = v[k];
    __syncthreads();
    if (tid < 12) {
      const int k = (int)tid;
      float r = s_red[k][0];
      for (int j = 1; j < kFusedWaves; ++j) r = (k % 6) < 3 ? fminf(r, s_red[k][j]) : fmaxf(r, s_red[k][j]);
      s_cb[k] = r;
      cb_out[k] = r;
    }
    __syncthreads();
  }
  RT_BT(1);
  // 2. Morton codes (k_morton)
  for (uint32_t i = tid; i < n; i += kFusedThreads) {
    const float* b = primbox + (size_t)i * 6;
    uint32_t q[3];
    for (int k = 0; k < 3; ++k) {
      const float ext = s_cb[3 + k] - s_cb[k];
      const float inv = ext > 0.0f ? 1.0f / ext : 0.0f;
      const float c = (b[k] + b[3 + k]) * 0.5f;
      q[k] = quantize10(c, s_cb[k], inv);
    }
    keyA[i] = (expand_bits10(q[0]) << 2) | (expand_bits10(q[1]) << 1) | expand_bits10(q[2]);
    valA[i] = i;
  }
  // 3. radix sort, 4 passes: A -> B -> A -> B -> A
  {
    const uint32_t chunk = (((n + kFusedWaves - 1) / kFusedWaves) + 63u) & ~63u;  // keys per wave
    const uint32_t c0 = w * chunk, c1 = min(c0 + chunk, n);
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64u - lane));
    uint32_t *kin = keyA, *vin = valA, *kout = keyB, *vout = valB;
    for (int pass = 0; pass < 4; ++pass) {
      const int shift = pass * 8;
      for (uint32_t k = tid; k < 256u * kFusedWaves; k += kFusedThreads) cnt[k] = 0;
      __syncthreads();
      // counts of each digit in this wave's chunk (one writer per (digit, wave): the rank-0 lane)
      for (uint32_t b = c0; b < c1; b += 64) {
        const uint32_t i = b + lane;
        const bool valid = i < c1;
        const uint32_t digit = valid ? (kin[i] >> shift) & 255u : 0u;
        uint64_t peers = __ballot(valid);
        for (int q = 0; q < 8; ++q) {
          const bool bit = (digit >> q) & 1u;
          const uint64_t m = __ballot(valid && bit);
          peers &= bit ? m : ~m;
        }
        if (valid && (peers & lt) == 0) cnt[w * 256u + digit] += (uint32_t)__popcll(peers);
      }
      __syncthreads();
      // exclusive scan over (digit, wave): 4 consecutive entries per thread
      {
        uint32_t e[4], s = 0;
        for (int q = 0; q < 4; ++q) {
          const uint32_t si = tid * 4 + q;  // scan order: digit-major, wave-minor
          e[q] = cnt[(si % kFusedWaves) * 256u + si / kFusedWaves];
          s += e[q];
        }
        uint32_t tot;
        uint32_t run = block_excl_scan(s, s_w, &tot);
        for (int q = 0; q < 4; ++q) {
          const uint32_t si = tid * 4 + q;
          cnt[(si % kFusedWaves) * 256u + si / kFusedWaves] = run;
          run += e[q];
        }
      }
      __syncthreads();
      // stable scatter: the wave's rounds in order, lanes in order within a round
      for (uint32_t b = c0; b < c1; b += 64) {
        const uint32_t i = b + lane;
        const bool valid = i < c1;
        const uint32_t key = valid ? kin[i] : 0u, val = valid ? vin[i] : 0u;
        const uint32_t digit = (key >> shift) & 255u;
        uint64_t peers = __ballot(valid);
        for (int q = 0; q < 8; ++q) {
          const bool bit = (digit >> q) & 1u;
          const uint64_t m = __ballot(valid && bit);
          peers &= bit ? m : ~m;
        }
        const uint32_t rank = (uint32_t)__popcll(peers & lt);
        const uint32_t base = valid ? cnt[w * 256u + digit] : 0u;  // every lane reads before the update
        if (valid) {
          kout[base + rank] = key;
          vout[base + rank] = val;
        }
        if (valid && rank == 0) cnt[w * 256u + digit] = base + (uint32_t)__popcll(peers);
      }
      __syncthreads();
      uint32_t* t = kin;
      kin = kout;
      kout = t;
      t = vin;
      vin = vout;
      vout = t;
    }
  }
  RT_BT(2);
  // sorted permutation (values A) out; Karras from keys A
  for (uint32_t i = tid; i < n; i += kFusedThreads) sorted[i] = valA[i];
  __syncthreads();  // values A and buffers B take the hierarchy: parents of internal nodes, children
  int* s_pint = (int*)s_mem + kFusedMax;
  int* s_child = (int*)s_mem + 2 * kFusedMax;
  if (n == 1) {
    if (tid == 0) {  // k_single
      BinNode nd;
      for (int k = 0; k < 3; ++k) {
        nd.lo0[k] = nd.lo1[k] = primbox[k];
        nd.hi0[k] = nd.hi1[k] = primbox[3 + k];
      }
      nd.c0 = ~0;
      nd.c1 = kEmptyChild;
      nd.pad0 = nd.pad1 = 0;
      bin[0] = nd;
    }
  } else {
    // 4. Karras (k_karras)
    for (int i = (int)tid; i < (int)n - 1; i += kFusedThreads) {
      const int nn = (int)n;
      const int d = (delta_lds(keyA, nn, i, i + 1) - delta_lds(keyA, nn, i, i - 1)) >= 0 ? 1 : -1;
      const int dmin = delta_lds(keyA, nn, i, i - d);
      int lmax = 2;
      while (delta_lds(keyA, nn, i, i + lmax * d) > dmin) lmax <<= 1;
      int l = 0;
      for (int t = lmax >> 1; t >= 1; t >>= 1)
        if (delta_lds(keyA, nn, i, i + (l + t) * d) > dmin) l += t;
      const int j = i + l * d;
      const int dnode = delta_lds(keyA, nn, i, j);
      int s = 0, t = l;
      while (true) {
        t = (t + 1) >> 1;
        if (delta_lds(keyA, nn, i, i + (s + t) * d) > dnode) s += t;
        if (t <= 1) break;
      }
      const int gamma = i + s * d + (d < 0 ? d : 0);
      const int lo = i < j ? i : j, hi = i < j ? j : i;
      const int left = (lo == gamma) ? ~gamma : gamma;
      const int right = (hi == gamma + 1) ? ~(gamma + 1) : gamma + 1;
      s_child[2 * i] = left;
      s_child[2 * i + 1] = right;
      if (left >= 0) s_pint[left] = i; else pleaf[~left] = i;
      if (right >= 0) s_pint[right] = i; else pleaf[~right] = i;
      if (i == 0) s_pint[0] = -1;
    }
  RT_BT(3);
    __syncthreads();  // keys no longer needed: the arrival flags take their words
    uint32_t* flags = s_mem;
    for (uint32_t i = tid; i < n - 1; i += kFusedThreads) flags[i] = 0;
    __syncthreads();
    // 5. refit + collapse DP (k_refit): the second arrival at a node computes it. Hand-off inside
    // the workgroup: the child's box / DP stores complete (vmcnt(0)), then the LDS counter.
    for (uint32_t i = tid; i < n; i += kFusedThreads) {
      int node = pleaf[i];
      while (node >= 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t old = __hip_atomic_fetch_add(&flags[node], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (old == 0) break;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        float a[6], b[6];
        const int ca = s_child[2 * node], cbb = s_child[2 * node + 1];
        load_box(ca, nbox, primbox, sorted, a);
        load_box(cbb, nbox, primbox, sorted, b);
        float bb[6];
        for (int k = 0; k < 3; ++k) {
          bb[k] = fminf(a[k], b[k]);
          bb[3 + k] = fmaxf(a[3 + k], b[3 + k]);
        }
        float* o = nbox + (size_t)node * 6;
        for (int k = 0; k < 6; ++k) o[k] = bb[k];
        if (dpc) sah_dp(node, bb, ca, cbb, dpc, dps);
        node = s_pint[node];
      }
    }
    __syncthreads();
  RT_BT(4);
    // 6. pack (k_pack)
    for (int i = (int)tid; i < (int)n - 1; i += kFusedThreads) {
      BinNode nd;
      int c[2] = {s_child[2 * i], s_child[2 * i + 1]};
      float b[2][6];
      for (int k = 0; k < 2; ++k) load_box(c[k], nbox, primbox, sorted, b[k]);
      for (int k = 0; k < 3; ++k) {
        nd.lo0[k] = b[0][k];
        nd.hi0[k] = b[0][3 + k];
        nd.lo1[k] = b[1][k];
        nd.hi1[k] = b[1][3 + k];
      }
      for (int k = 0; k < 2; ++k)
        if (c[k] < 0 && leaf_ref_is_prim) c[k] = ~(int)sorted[~c[k]];
      nd.c0 = c[0];
      nd.c1 = c[1];
      nd.pad0 = nd.pad1 = 0;
      bin[i] = nd;
    }
  }
  __syncthreads();
  RT_BT(5);
  RT_BT(6);
  // 8. collapse into BFS-ordered 4-wide nodes (k_collapse); level lists and stack sums in LDS
  {
    int* cur = (int*)s_mem;
    int* nxt = (int*)s_mem + kFusedMax;
    int* ps = (int*)s_mem + 2 * kFusedMax;
    if (tid == 0) {
      cur[0] = 0;
      ps[0] = 0;
      s_maxstack = 0;
    }
    __syncthreads();
    int lmax = 0, cur_n = 1, base = 0, depth = 0;
    while (cur_n > 0) {
      ++depth;
      int next_total = 0;
      for (int cs = 0; cs < cur_n; cs += kFusedThreads) {
        const int i = cs + (int)tid;
        const bool valid = i < cur_n;
        int ref[4];
        float box[4][6];
        int cnt4 = 0;
        if (valid) {
          if (dpc)  // the DP expansion of this wide node's root, in registers (no k_dp_expand pass)
            cnt4 = wide_slots_dp(bin, dpc, dps, cur[i], ref, box, !leaf_ref_is_prim);
          else {
            cnt4 = gather4(bin, cur[i], ref, box);
            for (int j = cnt4; j < 4; ++j) ref[j] = kEmptyChild;
            if (!leaf_ref_is_prim) inner_first(ref, box);
          }
        }
        uint32_t m = 0;
        for (int j = 0; j < cnt4; ++j) m += ref[j] >= 0;
        uint32_t chunk_total;
        const int excl = (int)block_excl_scan(m, s_w, &chunk_total);
        if (valid) {
          Bvh4Node nd;
          int o = excl;
          const int below = ps[base + i] + cnt4 - 1;
          lmax = below > lmax ? below : lmax;
          uint32_t nvalid = 0, inner = 0;
          nd.first_inner = 0;
          for (int j = 0; j < 4; ++j) {
            const float inf = __builtin_inff();
            float b6[6] = {inf, inf, inf, inf, inf, inf};
            int32_t r = kEmptyChild;
            if (j < cnt4 && ref[j] != kEmptyChild) {
              ++nvalid;
              for (int a = 0; a < 6; ++a) b6[a] = box[j][a];
              if (ref[j] >= 0) {
                const int pos = next_total + o;
                nxt[pos] = ref[j];
                r = base + cur_n + pos;
                ps[r] = below;
                if (o == excl) nd.first_inner = r;
                inner |= 1u << j;
                ++o;
              } else {
                r = ref[j];
              }
            }
            nd.lox[j] = b6[0];
            nd.loy[j] = b6[1];
            nd.loz[j] = b6[2];
            nd.hix[j] = b6[3];
            nd.hiy[j] = b6[4];
            nd.hiz[j] = b6[5];
            nd.child[j] = r;
          }
          nd.count = nvalid;
          nd.inner_mask = inner;
          nd.entry_base = ((uint32_t)nd.first_inner << 8) | (inner << 4);
          out[base + i] = nd;
        }
        next_total += (int)chunk_total;
      }
      __syncthreads();  // the next level reads nxt / ps
      int* t = cur;
      cur = nxt;
      nxt = t;
      base += cur_n;
      cur_n = next_total;
    }
    atomicMax(&s_maxstack, lmax);
    __syncthreads();
    if (tid == 0) {
      info[0] = (uint32_t)base;
      info[1] = (uint32_t)depth;
      info[2] = (uint32_t)s_maxstack;
    }
  }
  RT_BT(7);
  // 9. triangles into leaf order (k_tri_reorder)
  if (tri_in)
    for (uint32_t i = tid; i < n; i += kFusedThreads) tri_out[i] = tri_in[sorted[i]];
#if RT_BUILD_TIMING
  RT_BT(8);
  if (tid == 0)
    printf("k_build_small n=%u cycles: bounds %lu morton+sort %lu karras %lu refit %lu pack %lu dpexp %lu collapse %lu reorder %lu\n",
           n, bt[1] - bt[0], bt[2] - bt[1], bt[3] - bt[2], bt[4] - bt[3], bt[5] - bt[4], bt[6] - bt[5], bt[7] - bt[6],
           bt[8] - bt[7]);
#endif
#undef RT_BT
}

// ------------------------------------------------------------------------------------------
// Four-launch build for RT_MID_MIN_N <= n <= kMidMax (the teapot / rabbit BLASes, every TLAS of
// the configs) instead of ~20 launches, none of them a long single-workgroup pipeline:
//   k_mid_rank       bounds + Morton codes + sort by RANK, one launch: every workgroup reduces the
//                    bounds of all n boxes itself (exact min / max: any order gives the same
//                    floats), holds all n keys in LDS, and ranks 64 of them with 16 waves splitting
//                    the j range: the stable order of key64 = morton << 32 | index is
//                    rank(i) = #{j : key64_j < key64_i}. The scatter by rank also writes the
//                    triangles in leaf order.
//   k_mid_tree       hierarchy + refit + SAH DP + pack in ONE bottom-up pass (Apetrei 2014,
//                    agglomerative LBVH): a node [l, r] is the left child of the split at r when
//                    delta(r) > delta(l - 1), else the right child of the split at l - 1, so a leaf's
//                    thread climbs without parent pointers. The binary radix tree over distinct keys
//                    is unique, so this is Karras' tree (internal nodes numbered by split position
//                    instead; the collapse output does not depend on the numbering). A workgroup
//                    owns a block of S leaves and completes every node whose range stays inside it,
//                    hand-offs through LDS. Whether a parent stays inside is decided from its split
//                    s alone (its range is the keys sharing delta(s) prefix bits with key s: inside
//                    iff lcp(s, B - 1) < delta(s) and lcp(s, B + S) < delta(s)), so both arrivals
//                    agree; a child whose parent leaves the block goes to the frontier list.
//   k_mid_expand     the DP expansion (wide_slots_dp) of every node built so far, in parallel
//   k_mid_collapse   one workgroup: the top of the tree climbed from the frontier with LDS hand-
//                    offs (the nodes that cross block boundaries: at most (blocks - 1) x 64, the
//                    key64 bit length bounding the depth), their expansions, then the BFS numbering
//                    level by level over 16-bit child lists in LDS, every 4-wide node written in
//                    parallel.
// The device-scope arrival protocol of k_refit (a write-through payload, a wait for its
// acknowledgement and an agent-scope atomic per level: ~3 memory round trips) is not used: the
// block-crossing chains from the block boundaries to the root were the critical path with it.
// ------------------------------------------------------------------------------------------
#define RT_KCONST __attribute__((address_space(4)))
constexpr uint32_t kMidMax = 8192;
constexpr int kMidBlock = 1024;       // leaves per k_mid_tree workgroup
constexpr int kMidTopSlots = 1024;    // top-climb payload slots: >= 2 x (kMidMax / kMidBlock - 1) x 64
constexpr uint16_t kMidLeaf = 0xfffeu, kMidEmpty = 0xffffu;
constexpr uint32_t kDpsUnbuilt = 0xffffffffu;  // dps of a node k_mid_tree left to the collapse
static_assert(kMidTopSlots >= 2 * (kMidMax / kMidBlock - 1) * 64, "top-climb slots");

struct MidSlot {  // a child's hand-off record: box, DP costs, ref, range
  float b[6];
  float d[4];
  int32_t ref, l, r, pad;
};

__device__ __forceinline__ int lcp64(uint64_t a, uint64_t b) { return __clzll(a ^ b); }

// Builds the parent at split s from its two children (a = this thread's node, o = the sibling's
// record; `left`: a is the left child): BinNode, DP (k_refit / k_pack arithmetic, left child first),
// and the parent's box / DP / range back into a.
__device__ __forceinline__ void mid_join(int s, bool left, MidSlot& a, const MidSlot& o, BinNode* __restrict__ bin,
                                         float4* __restrict__ dpc, uint32_t* __restrict__ dps) {
  const MidSlot& L = left ? a : o;
  const MidSlot& R = left ? o : a;
  BinNode nd;
  float bb[6];
  for (int k = 0; k < 3; ++k) {
    nd.lo0[k] = L.b[k];
    nd.hi0[k] = L.b[3 + k];
    nd.lo1[k] = R.b[k];
    nd.hi1[k] = R.b[3 + k];
    bb[k] = fminf(L.b[k], R.b[k]);
    bb[3 + k] = fmaxf(L.b[3 + k], R.b[3 + k]);
  }
  nd.c0 = L.ref;
  nd.c1 = R.ref;
  nd.pad0 = nd.pad1 = 0;
  float4 dc;
  uint32_t sj;
  sah_dp_vals(bb, make_float4(L.d[0], L.d[1], L.d[2], L.d[3]), make_float4(R.d[0], R.d[1], R.d[2], R.d[3]), dc, sj);
  const int nl = L.l, nr = R.r;
  bin[s] = nd;
  dpc[s] = dc;
  dps[s] = sj;
  for (int k = 0; k < 6; ++k) a.b[k] = bb[k];
  a.d[0] = dc.x;
  a.d[1] = dc.y;
  a.d[2] = dc.z;
  a.d[3] = dc.w;
  a.ref = s;
  a.l = nl;
  a.r = nr;
}

__global__ __launch_bounds__(1024) void k_mid_rank(const float* __restrict__ primbox, uint32_t n,
                                                   float* __restrict__ cb_out, uint64_t* keys64,
                                                   uint32_t* __restrict__ keys_sorted, uint32_t* __restrict__ sorted,
                                                   float* __restrict__ sbox,
                                                   uint32_t* __restrict__ dps, uint32_t* __restrict__ info,
                                                   const TriRec* __restrict__ tri_in, TriRec* __restrict__ tri_out) {
  __shared__ uint32_t s_part[16][64];
  __shared__ float s_red[12][16];
  __shared__ float s_cb[12];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
  constexpr int kPer = kMidMax / 1024;
  float bx[kPer][6];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {  // past n: copies of the last box (the min / max do not change)
    const uint32_t i = min(tid + 1024u * q, n - 1u);
#pragma unroll
    for (int k = 0; k < 6; ++k) bx[q][k] = primbox[(size_t)i * 6 + k];
  }
  {  // bounds (k_bounds' values: exact min / max)
    float v[12];
    for (int k = 0; k < 3; ++k) {
      v[k] = INFINITY;
      v[3 + k] = -INFINITY;
      v[6 + k] = INFINITY;
      v[9 + k] = -INFINITY;
    }
#pragma unroll
    for (int q = 0; q < kPer; ++q)
      for (int k = 0; k < 3; ++k) {
          const float c = (bx[q][k] + bx[q][3 + k]) * 0.5f;
          v[k] = fminf(v[k], c);
          v[3 + k] = fmaxf(v[3 + k], c);
          v[6 + k] = fminf(v[6 + k], bx[q][k]);
          v[9 + k] = fmaxf(v[9 + k], bx[q][3 + k]);
        }
    for (int off = 32; off >= 1; off >>= 1)
      for (int k = 0; k < 12; ++k) {
        const float o = __shfl_xor(v[k], off, 64);
        v[k] = (k % 6) < 3 ? fminf(v[k], o) : fmaxf(v[k], o);
      }
    if (lane == 0)
      for (int k = 0; k < 12; ++k) s_red[k][w] = v[k];
    __syncthreads();
    if (tid < 12) {
      const int k = (int)tid;
      float r = s_red[k][0];
      for (int j = 1; j < 16; ++j) r = (k % 6) < 3 ? fminf(r, s_red[k][j]) : fmaxf(r, s_red[k][j]);
      s_cb[k] = r;
      if (blockIdx.x == 0) cb_out[k] = r;
    }
    if (blockIdx.x == 0 && tid == 12) info[4] = 0u;  // k_mid_tree's frontier count
    __syncthreads();
  }
  float lo[3], inv[3];
  for (int k = 0; k < 3; ++k) {  // k_morton's quantisation, operation for operation
    const float ext = s_cb[3 + k] - s_cb[k];
    inv[k] = ext > 0.0f ? 1.0f / ext : 0.0f;
    lo[k] = s_cb[k];
  }
  // every workgroup computes every key; all of them store the same values to keys64 (a benign
  // race of identical data), read back through the scalar cache: the j keys are wave-uniform, so
  // they travel as SGPR operands instead of through the LDS / L1 return path to 64 lanes
  uint64_t ki = ~0ull;
  const uint32_t iq = blockIdx.x * 64u + lane;  // this lane's key
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const uint32_t i = tid + 1024u * q;
    if (i < n) {
      uint32_t c[3];
      for (int k = 0; k < 3; ++k) c[k] = quantize10((bx[q][k] + bx[q][3 + k]) * 0.5f, lo[k], inv[k]);
      const uint32_t code = (expand_bits10(c[0]) << 2) | (expand_bits10(c[1]) << 1) | expand_bits10(c[2]);
      keys64[i] = ((uint64_t)code << 32) | i;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const RT_KCONST uint64_t* kc = (const RT_KCONST uint64_t*)keys64;
  asm volatile("" : "+s"(kc));  // the scalar loads stay behind the barrier
  if (iq < n) ki = kc[iq];
  const uint32_t wu = (uint32_t)__builtin_amdgcn_readfirstlane((int)w);  // wave-uniform: scalar j loop
  const uint32_t chunk = (((n + 15u) / 16u) + 31u) & ~31u, j0 = min(wu * chunk, n), j1 = min(j0 + chunk, n);
  uint32_t c = 0;
  uint32_t j = j0;
  typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
  for (; j + 32 <= j1; j += 32) {  // 8 keys per s_load_dwordx16, four loads in flight (the keys
                                   // were just written: scalar-cache misses, L2 latency each)
    u32x16 kv[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) kv[h] = *(const RT_KCONST u32x16*)(kc + j + 8 * h);
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
      for (int u = 0; u < 8; ++u) c += (((uint64_t)kv[h][2 * u + 1] << 32) | kv[h][2 * u]) < ki ? 1u : 0u;
  }
  for (; j < j1; ++j) c += kc[j] < ki ? 1u : 0u;
  s_part[w][lane] = c;
  __syncthreads();
  const uint32_t i = iq;
  if (i >= n) return;
  if (w == 0) {
    uint32_t rank = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) rank += s_part[q][lane];
    keys_sorted[rank] = (uint32_t)(ki >> 32);
    sorted[rank] = i;
    for (int k = 0; k < 6; ++k) sbox[(size_t)rank * 6 + k] = primbox[(size_t)i * 6 + k];
    if (tri_out) tri_out[rank] = tri_in[i];
  } else if (w == 1 && i + 1 < n) {
    dps[i] = kDpsUnbuilt;  // overwritten by whichever kernel builds split i
  }
}

__global__ __launch_bounds__(kMidBlock) void k_mid_tree(uint32_t n, const uint32_t* __restrict__ keys_sorted,
                                                        const uint32_t* __restrict__ sorted,
                                                        const float* __restrict__ sbox, bool leaf_ref_is_prim,
                                                        BinNode* __restrict__ bin, float4* __restrict__ dpc,
                                                        uint32_t* __restrict__ dps, MidSlot* __restrict__ frontier,
                                                        uint32_t* __restrict__ info) {
  __shared__ uint64_t s_k[kMidBlock + 2];  // keys B - 1 .. B + S
  __shared__ uint32_t s_flag[kMidBlock];
  __shared__ MidSlot s_slot[kMidBlock];   // by position: the left child of split s at s, the right at s + 1
  const uint32_t S = kMidBlock, B = blockIdx.x * S, tid = threadIdx.x;
  for (uint32_t k = tid; k < S + 2; k += S) {
    const int64_t p = (int64_t)B - 1 + (int64_t)k;
    s_k[k] = (p >= 0 && p < (int64_t)n) ? (((uint64_t)keys_sorted[p] << 32) | (uint64_t)p) : 0ull;
  }
  s_flag[tid] = 0u;
  __syncthreads();
  const uint32_t i = B + tid;
  if (i >= n) return;
  MidSlot a;
  {
    const uint32_t prim = sorted[i];
    const float* p = sbox + (size_t)i * 6;  // the leaf boxes in leaf order (k_mid_rank)
    for (int k = 0; k < 6; ++k) a.b[k] = p[k];
    for (int k = 0; k < 4; ++k) a.d[k] = 0.0f;
    a.ref = leaf_ref_is_prim ? ~(int)prim : ~(int)i;
    a.l = a.r = (int)i;
    a.pad = 0;
  }
  const int ib = (int)B;
  const uint64_t kb0 = s_k[0], kb1 = s_k[S + 1];  // keys B - 1 and B + S
  while (!(a.l == 0 && a.r == (int)n - 1)) {
    // the four keys around the node in one LDS round trip (past the ends: unused zeros)
    const uint64_t klm = s_k[a.l - ib], kl = s_k[a.l - ib + 1], kr = s_k[a.r - ib + 1], krp = s_k[a.r - ib + 2];
    const int dl = a.l > 0 ? lcp64(klm, kl) : -1;
    const int dr = a.r < (int)n - 1 ? lcp64(kr, krp) : -1;
    const bool left = dr > dl;  // this node is the left child of the split at r
    const int s = left ? a.r : a.l - 1;
    const int q = left ? dr : dl;
    const uint64_t ks = left ? kr : klm;  // key s
    const bool inside = s >= ib && s + 1 < ib + (int)S && (B == 0 || lcp64(ks, kb0) < q) &&
                        (B + S >= n || lcp64(ks, kb1) < q);
    if (!inside) {  // the parent crosses the block: the collapse workgroup climbs on from here
      const uint32_t f = __hip_atomic_fetch_add(&info[4], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      frontier[f] = a;
      return;
    }
    const int pos = (left ? s : s + 1) - ib;
    s_slot[pos] = a;
    // LDS executes one wave's operations in order and the sibling's record is read only after its
    // arrival was observed: a relaxed LDS atomic between compiler barriers orders the hand-off. An
    // acquire / release atomic would also wait for this thread's outstanding HBM stores (bin, DP)
    // at every level.
    asm volatile("" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(&s_flag[s - ib], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
    if (old == 0) return;
    const MidSlot o = s_slot[(left ? s + 1 : s) - ib];
    mid_join(s, left, a, o, bin, dpc, dps);
  }
  info[3] = (uint32_t)a.ref;  // the whole tree inside one block: the root's binary index
}

__global__ void k_mid_expand(int nbin, const BinNode* __restrict__ bin, const float4* __restrict__ dpc,
                             const uint32_t* __restrict__ dps, Exp4* __restrict__ exp, uint2* __restrict__ e16,
                             bool blas) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nbin || dps[i] == kDpsUnbuilt) return;  // top nodes: expanded by k_mid_collapse
  Exp4 e;
  e.cnt = wide_slots_dp(bin, dpc, dps, i, e.ref, e.box, blas);
  e.pad[0] = e.pad[1] = e.pad[2] = 0;
  exp[i] = e;
  uint32_t h[4];
  for (int j = 0; j < 4; ++j) h[j] = j >= e.cnt ? kMidEmpty : e.ref[j] >= 0 ? (uint32_t)e.ref[j] : kMidLeaf;
  e16[i] = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
}

__global__ __launch_bounds__(1024) void k_mid_collapse(uint32_t n, const uint32_t* __restrict__ keys_sorted,
                                                       const MidSlot* __restrict__ frontier, BinNode* bin,
                                                       float4* dpc, uint32_t* dps, Exp4* exp,
                                                       const uint2* __restrict__ e16, uint16_t* __restrict__ order_out,
                                                       uint16_t* __restrict__ bfs_out, uint32_t* __restrict__ info,
                                                       bool blas) {
  // phase A (top climb): keys | arrival words | payload slots; afterwards the same bytes hold the
  // 16-bit child lists, the BFS order / index maps and the stack sums
  constexpr size_t kA = kMidMax * 8 + kMidMax * 4 + kMidTopSlots * sizeof(MidSlot);
  constexpr size_t kD = kMidMax * 8 + 3 * kMidMax * 2;
  __shared__ __attribute__((aligned(16))) unsigned char s_raw[kA > kD ? kA : kD];
  __shared__ uint16_t s_top[kMidTopSlots];
  __shared__ uint32_t s_ntop, s_nslot, s_root;
  __shared__ uint32_t s_w[2 * kFusedWaves];
  __shared__ int s_maxstack;
  const int tid = (int)threadIdx.x;
  const int nbin = (int)n - 1;
#if RT_BUILD_TIMING
  uint64_t bt[4];
  bt[0] = __builtin_amdgcn_s_memtime();
#define RT_BT(k) bt[k] = __builtin_amdgcn_s_memtime()
#else
#define RT_BT(k) (void)0
#endif
  const uint32_t nf = info[4];
  // the child lists of every node k_mid_expand built, loaded now (into registers: the LDS they go to
  // holds the top climb's keys and slots first), in flight during the top climb
  constexpr int kPer = kMidMax / 1024;
  uint2 ev[kPer];
#pragma unroll
  for (int q = 0; q < kPer; ++q) ev[q] = e16[min(tid + 1024 * q, nbin - 1)];
  if (nf > 0) {
    uint64_t* s_k = (uint64_t*)s_raw;
    uint32_t* s_arr = (uint32_t*)(s_raw + kMidMax * 8);
    MidSlot* s_pay = (MidSlot*)(s_raw + kMidMax * 8 + kMidMax * 4);
    MidSlot a0;
    if ((uint32_t)tid < nf) a0 = frontier[tid];
    for (int k = tid; k < (int)n; k += 1024) s_k[k] = ((uint64_t)keys_sorted[k] << 32) | (uint64_t)k;
    for (int k = tid; k < nbin; k += 1024) s_arr[k] = 0u;
    if (tid == 0) s_ntop = s_nslot = 0u;
    __syncthreads();
    for (uint32_t f = (uint32_t)tid; f < nf; f += 1024u) {
      MidSlot a = f == (uint32_t)tid ? a0 : frontier[f];
      while (!(a.l == 0 && a.r == (int)n - 1)) {
        const uint64_t klm = s_k[max(a.l - 1, 0)], kl = s_k[a.l], kr = s_k[a.r], krp = s_k[min(a.r + 1, (int)n - 1)];
        const int dl = a.l > 0 ? lcp64(klm, kl) : -1;
        const int dr = a.r < (int)n - 1 ? lcp64(kr, krp) : -1;
        const bool left = dr > dl;
        const int s = left ? a.r : a.l - 1;
        // each arrival parks its record in a fresh slot and swaps the slot (+1) into the split's
        // word: the second arrival gets the first's slot back
        const uint32_t mine = __hip_atomic_fetch_add(&s_nslot, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        s_pay[mine] = a;
        asm volatile("" ::: "memory");  // LDS order suffices (see k_mid_tree): no wait for HBM stores
        const uint32_t other =
            __hip_atomic_exchange(&s_arr[s], mine + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        asm volatile("" ::: "memory");
        if (other == 0u) break;
        const MidSlot o = s_pay[other - 1u];
        mid_join(s, left, a, o, bin, dpc, dps);
        s_top[__hip_atomic_fetch_add(&s_ntop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)] = (uint16_t)s;
        if (a.l == 0 && a.r == (int)n - 1) s_root = (uint32_t)s;
#if RT_BUILD_TIMING
        if (a.l == 0 && a.r == (int)n - 1)
          printf("  top climb: root thread %d done at %lu (start %lu)\n", tid, __builtin_amdgcn_s_memtime() - bt[0], 0ul);
#endif
      }
    }
    __threadfence_block();
    __syncthreads();
  } else if (tid == 0) {
    s_ntop = 0u;
    s_root = info[3];
  }
  __syncthreads();
  RT_BT(1);
  uint2* s_e = (uint2*)s_raw;                                  // per binary node: its wide node's slot refs
  uint16_t* s_order = (uint16_t*)(s_raw + kMidMax * 8);        // BFS index -> binary node
  uint16_t* s_bfs = s_order + kMidMax;                         // binary node -> BFS index
  uint16_t* s_ps = s_bfs + kMidMax;                            // BFS index -> stack entries below
#pragma unroll
  for (int q = 0; q < kPer; ++q)
    if (tid + 1024 * q < nbin) s_e[tid + 1024 * q] = ev[q];
  const int ntop = (int)s_ntop;
  __syncthreads();
  // phase B: expansions of the top nodes (their descendants are all built now)
  for (int k = tid; k < ntop; k += 1024) {
    const int sn = (int)s_top[k];
    Exp4 e;
    e.cnt = wide_slots_dp(bin, dpc, dps, sn, e.ref, e.box, blas);
    e.pad[0] = e.pad[1] = e.pad[2] = 0;
    exp[sn] = e;
    uint32_t h[4];
    for (int j = 0; j < 4; ++j) h[j] = j >= e.cnt ? kMidEmpty : e.ref[j] >= 0 ? (uint32_t)e.ref[j] : kMidLeaf;
    s_e[sn] = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
  }
  const int root = min((int)s_root, nbin - 1);  // (a root outside the tree would be a bug)
  __threadfence_block();
  __syncthreads();
  RT_BT(2);
  if (tid == 0) {
    s_order[0] = (uint16_t)root;
    s_bfs[root] = 0;
    s_ps[0] = 0;
    s_maxstack = 0;
  }
  __syncthreads();
  // phase C: BFS numbering, level by level, two barriers per level. A thread takes `per` consecutive
  // nodes of the level; the exclusive sum of their internal-child counts (<= 32: six bits) is
  // formed from one ballot per bit (popcount of the lower lanes), the waves' totals through LDS.
  int lmax = 0, cur_n = 1, base = 0, depth = 0;
#if RT_BUILD_TIMING
  uint64_t lvt[16];
  lvt[0] = __builtin_amdgcn_s_memtime();
#endif
  const uint32_t lane = (uint32_t)tid & 63u, wv = (uint32_t)tid >> 6;
  const uint64_t lower = lane == 0 ? 0ull : (~0ull >> (64u - lane));
  while (cur_n > 0) {
    const int per = (cur_n + 1023) / 1024;  // <= 8
    const int i0 = min(tid * per, cur_n), i1 = min(i0 + per, cur_n);
    uint32_t msum = 0;
    for (int i = i0; i < i1; ++i) {
      const uint2 e = s_e[s_order[base + i]];
      msum += ((e.x & 0xffffu) < kMidLeaf ? 1u : 0u) + ((e.x >> 16) < kMidLeaf ? 1u : 0u) +
              ((e.y & 0xffffu) < kMidLeaf ? 1u : 0u) + ((e.y >> 16) < kMidLeaf ? 1u : 0u);
    }
    uint32_t pre = 0, wtot = 0;
#pragma unroll
    for (int bit = 0; bit < 6; ++bit) {
      const uint64_t bal = __ballot((msum >> bit) & 1u);
      pre += (uint32_t)__popcll(bal & lower) << bit;
      wtot += (uint32_t)__popcll(bal) << bit;
    }
    uint32_t* s_wl = s_w + (depth & 1) * kFusedWaves;  // double-buffered: no barrier before the write
    if (lane == 0) s_wl[wv] = wtot;
    __syncthreads();
    uint32_t woff = 0, total = 0;
#pragma unroll
    for (int k = 0; k < kFusedWaves; ++k) {
      const uint32_t c = s_wl[k];
      woff += (uint32_t)k < wv ? c : 0u;
      total += c;
    }
    int o = base + cur_n + (int)(woff + pre);
    for (int i = i0; i < i1; ++i) {
      const uint2 e = s_e[s_order[base + i]];
      const uint32_t h[4] = {e.x & 0xffffu, e.x >> 16, e.y & 0xffffu, e.y >> 16};
      uint32_t cnt = 0;
      for (int j = 0; j < 4; ++j) cnt += h[j] != kMidEmpty ? 1u : 0u;
      const int below = (int)s_ps[base + i] + (int)cnt - 1;
      lmax = below > lmax ? below : lmax;
      for (int j = 0; j < 4; ++j)
        if (h[j] < kMidLeaf) {
          s_order[o] = (uint16_t)h[j];
          s_bfs[h[j]] = (uint16_t)o;
          s_ps[o] = (uint16_t)below;
          ++o;
        }
    }
    ++depth;
    __syncthreads();
#if RT_BUILD_TIMING
    if (depth < 16) lvt[depth] = __builtin_amdgcn_s_memtime();
#endif
    base += cur_n;
    cur_n = (int)total;
  }
  RT_BT(3);
  // the node writes run in k_mid_write (many workgroups): BFS order and index maps to HBM
  for (int k = tid; k < base; k += 1024) order_out[k] = s_order[k];
  for (int k = tid; k < nbin; k += 1024) bfs_out[k] = s_bfs[k];
  atomicMax(&s_maxstack, lmax);
  __syncthreads();
  if (tid == 0) {
    info[0] = (uint32_t)base;
    info[1] = (uint32_t)depth;
    info[2] = (uint32_t)s_maxstack;
#if RT_BUILD_TIMING
    printf("k_mid_collapse n=%u frontier %u top %d levels %d cycles: top-climb %lu expand %lu bfs %lu\n", n, nf, ntop,
           depth, bt[1] - bt[0], bt[2] - bt[1], bt[3] - bt[2]);
    for (int k = 1; k < depth && k < 16; ++k) printf("  bfs level %d: %lu\n", k, lvt[k] - lvt[k - 1]);
#endif
  }
#undef RT_BT
}

// Every 4-wide node in parallel (BFS index k): its wide root's expansion with the slot refs mapped to
// BFS indices.
__global__ void k_mid_write(const Exp4* __restrict__ exp, const uint16_t* __restrict__ order,
                            const uint16_t* __restrict__ bfs, const uint32_t* __restrict__ info,
                            Bvh4Node* __restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (int)info[0]) return;
  const Exp4& e = exp[order[k]];
  Bvh4Node nd;
  uint32_t nvalid = 0, inner = 0;
  nd.first_inner = 0;
  for (int j = 0; j < 4; ++j) {
    const float inf = __builtin_inff();
    float b6[6] = {inf, inf, inf, inf, inf, inf};
    int32_t r = kEmptyChild;
    if (j < e.cnt && e.ref[j] != kEmptyChild) {
      ++nvalid;
      for (int q = 0; q < 6; ++q) b6[q] = e.box[j][q];
      if (e.ref[j] >= 0) {
        r = (int32_t)bfs[e.ref[j]];
        if (!inner) nd.first_inner = r;
        inner |= 1u << j;
      } else {
        r = e.ref[j];
      }
    }
    nd.lox[j] = b6[0];
    nd.loy[j] = b6[1];
    nd.loz[j] = b6[2];
    nd.hix[j] = b6[3];
    nd.hiy[j] = b6[4];
    nd.hiz[j] = b6[5];
    nd.child[j] = r;
  }
  nd.count = nvalid;
  nd.inner_mask = inner;
  nd.entry_base = ((uint32_t)nd.first_inner << 8) | (inner << 4);
  out[k] = nd;
}

// ------------------------------------------------------------------------------------------
// One-launch build for 2 <= n <= kTinyMax (the TLASes and the plane BLAS of the configs): the
// k_mid_* stages in ONE 512-thread workgroup with every intermediate in LDS — rank sort, the
// Apetrei climb (the whole tree is one block: every hand-off in LDS), the binary nodes, their DP and
// expansions, the BFS numbering — and only the finished 4-wide nodes (and the triangle gather)
// written to HBM. Same arithmetic in the same order as k_mid_*: the identical tree.
// ------------------------------------------------------------------------------------------
constexpr uint32_t kTinyMax = 512;
constexpr int kTinyWaves = kTinyMax / 64;

// The 4-wide node for a wide root's expansion (ref / box / cnt), slot refs mapped to BFS indices.
__device__ __forceinline__ void write_wide_node(const int (&ref)[4], const float (&box)[4][6], int cnt,
                                                const uint16_t* bfs, Bvh4Node* __restrict__ out) {
  Bvh4Node nd;
  uint32_t nvalid = 0, inner = 0;
  nd.first_inner = 0;
  for (int j = 0; j < 4; ++j) {
    const float inf = __builtin_inff();
    float b6[6] = {inf, inf, inf, inf, inf, inf};
    int32_t r = kEmptyChild;
    if (j < cnt && ref[j] != kEmptyChild) {
      ++nvalid;
      for (int q = 0; q < 6; ++q) b6[q] = box[j][q];
      if (ref[j] >= 0) {
        r = (int32_t)bfs[ref[j]];
        if (!inner) nd.first_inner = r;
        inner |= 1u << j;
      } else {
        r = ref[j];
      }
    }
    nd.lox[j] = b6[0];
    nd.loy[j] = b6[1];
    nd.loz[j] = b6[2];
    nd.hix[j] = b6[3];
    nd.hiy[j] = b6[4];
    nd.hiz[j] = b6[5];
    nd.child[j] = r;
  }
  nd.count = nvalid;
  nd.inner_mask = inner;
  nd.entry_base = ((uint32_t)nd.first_inner << 8) | (inner << 4);
  *out = nd;
}

__global__ __launch_bounds__(kTinyMax) void k_build_tiny(const float* __restrict__ primbox, uint32_t n,
                                                         bool leaf_ref_is_prim, uint32_t* __restrict__ sorted,
                                                         float* __restrict__ cb_out, Bvh4Node* __restrict__ out,
                                                         uint32_t* __restrict__ info, const TriRec* __restrict__ tri_in,
                                                         TriRec* __restrict__ tri_out) {
  __shared__ uint64_t s_key[kTinyMax];   // key64 by primitive, then (s_skey) by leaf position
  __shared__ uint64_t s_skey[kTinyMax];
  __shared__ float s_lbox[kTinyMax][6];  // leaf boxes in leaf order
  __shared__ uint32_t s_lprim[kTinyMax];
  __shared__ uint32_t s_flag[kTinyMax];
  __shared__ MidSlot s_slot[kTinyMax];   // by position, as in k_mid_tree
  __shared__ BinNode s_bin[kTinyMax];
  __shared__ float4 s_dpc[kTinyMax];
  __shared__ uint32_t s_dps[kTinyMax];
  __shared__ uint2 s_e[kTinyMax];
  __shared__ uint16_t s_order[kTinyMax], s_bfs[kTinyMax], s_ps[kTinyMax];
  __shared__ float s_red[12][kTinyWaves];
  __shared__ float s_cb[12];
  __shared__ uint32_t s_w[2 * kTinyWaves];
  __shared__ int s_root, s_maxstack;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
  const int nbin = (int)n - 1;
  // 1. bounds (k_bounds' values) and keys
  float bx[6];
  {
    const uint32_t i = min(tid, n - 1u);  // past n: copies of the last box
    for (int k = 0; k < 6; ++k) bx[k] = primbox[(size_t)i * 6 + k];
    float v[12];
    for (int k = 0; k < 3; ++k) {
      const float c = (bx[k] + bx[3 + k]) * 0.5f;
      v[k] = c;
      v[3 + k] = c;
      v[6 + k] = bx[k];
      v[9 + k] = bx[3 + k];
    }
    for (int off = 32; off >= 1; off >>= 1)
      for (int k = 0; k < 12; ++k) {
        const float o = __shfl_xor(v[k], off, 64);
        v[k] = (k % 6) < 3 ? fminf(v[k], o) : fmaxf(v[k], o);
      }
    if (lane == 0)
      for (int k = 0; k < 12; ++k) s_red[k][w] = v[k];
    if (tid == 0) s_maxstack = 0;
    __syncthreads();
    if (tid < 12) {
      const int k = (int)tid;
      float r = s_red[k][0];
      for (int j = 1; j < kTinyWaves; ++j) r = (k % 6) < 3 ? fminf(r, s_red[k][j]) : fmaxf(r, s_red[k][j]);
      s_cb[k] = r;
      cb_out[k] = r;
    }
    __syncthreads();
  }
  if (tid < n) {
    uint32_t q[3];
    for (int k = 0; k < 3; ++k) {  // k_morton's quantisation, operation for operation
      const float ext = s_cb[3 + k] - s_cb[k];
      const float inv = ext > 0.0f ? 1.0f / ext : 0.0f;
      q[k] = quantize10((bx[k] + bx[3 + k]) * 0.5f, s_cb[k], inv);
    }
    const uint32_t code = (expand_bits10(q[0]) << 2) | (expand_bits10(q[1]) << 1) | expand_bits10(q[2]);
    s_key[tid] = ((uint64_t)code << 32) | tid;
  }
  s_flag[tid] = 0u;
  __syncthreads();
  // 2. rank sort (stable: key64 carries the index) and the scatter into leaf order
  if (tid < n) {
    const uint64_t ki = s_key[tid];
    uint32_t rank = 0;
    for (uint32_t j = 0; j < n; ++j) rank += s_key[j] < ki ? 1u : 0u;
    s_skey[rank] = ((ki >> 32) << 32) | rank;  // key64 of the sorted array: code << 32 | position
    for (int k = 0; k < 6; ++k) s_lbox[rank][k] = bx[k];
    s_lprim[rank] = tid;
    sorted[rank] = tid;
    if (tri_out) tri_out[rank] = tri_in[tid];
  }
  __syncthreads();
  // 3. the Apetrei climb, one block: every hand-off in LDS
  if (tid < n) {
    MidSlot a;
    for (int k = 0; k < 6; ++k) a.b[k] = s_lbox[tid][k];
    for (int k = 0; k < 4; ++k) a.d[k] = 0.0f;
    a.ref = leaf_ref_is_prim ? ~(int)s_lprim[tid] : ~(int)tid;
    a.l = a.r = (int)tid;
    a.pad = 0;
    while (!(a.l == 0 && a.r == nbin)) {
      const uint64_t klm = s_skey[max(a.l - 1, 0)], kl = s_skey[a.l], kr = s_skey[a.r], krp = s_skey[min(a.r + 1, nbin)];
      const int dl = a.l > 0 ? lcp64(klm, kl) : -1;
      const int dr = a.r < nbin ? lcp64(kr, krp) : -1;
      const bool left = dr > dl;
      const int s = left ? a.r : a.l - 1;
      s_slot[left ? s : s + 1] = a;
      asm volatile("" ::: "memory");  // LDS order suffices (k_mid_tree)
      const uint32_t old = __hip_atomic_fetch_add(&s_flag[s], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      asm volatile("" ::: "memory");
      if (old == 0) break;
      const MidSlot o = s_slot[left ? s + 1 : s];
      mid_join(s, left, a, o, s_bin, s_dpc, s_dps);
    }
    if (a.l == 0 && a.r == nbin) s_root = a.ref;
  }
  __syncthreads();
  // 4. expansions (child lists for the numbering; recomputed for the node writes)
  const bool blas = !leaf_ref_is_prim;
  for (int sn = (int)tid; sn < nbin; sn += kTinyMax) {
    int ref[4];
    float box[4][6];
    const int cnt = wide_slots_dp(s_bin, s_dpc, s_dps, sn, ref, box, blas);
    uint32_t h[4];
    for (int j = 0; j < 4; ++j) h[j] = j >= cnt ? kMidEmpty : ref[j] >= 0 ? (uint32_t)ref[j] : kMidLeaf;
    s_e[sn] = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
  }
  if (tid == 0) {
    s_order[0] = (uint16_t)s_root;
    s_bfs[s_root] = 0;
    s_ps[0] = 0;
  }
  __syncthreads();
  // 5. BFS numbering (k_mid_collapse phase C, one node per thread: a level holds < kTinyMax nodes)
  const uint64_t lower = lane == 0 ? 0ull : (~0ull >> (64u - lane));
  int lmax = 0, cur_n = 1, base = 0, depth = 0;
  while (cur_n > 0) {
    const bool valid = (int)tid < cur_n;
    uint32_t h[4] = {kMidEmpty, kMidEmpty, kMidEmpty, kMidEmpty};
    if (valid) {
      const uint2 e = s_e[s_order[base + tid]];
      h[0] = e.x & 0xffffu;
      h[1] = e.x >> 16;
      h[2] = e.y & 0xffffu;
      h[3] = e.y >> 16;
    }
    uint32_t m = 0, cnt = 0;
    for (int j = 0; j < 4; ++j) {
      m += h[j] < kMidLeaf ? 1u : 0u;
      cnt += h[j] != kMidEmpty ? 1u : 0u;
    }
    uint32_t pre = 0, wtot = 0;
#pragma unroll
    for (int bit = 0; bit < 3; ++bit) {
      const uint64_t bal = __ballot((m >> bit) & 1u);
      pre += (uint32_t)__popcll(bal & lower) << bit;
      wtot += (uint32_t)__popcll(bal) << bit;
    }
    uint32_t* s_wl = s_w + (depth & 1) * kTinyWaves;
    if (lane == 0) s_wl[w] = wtot;
    __syncthreads();
    uint32_t woff = 0, total = 0;
#pragma unroll
    for (int k = 0; k < kTinyWaves; ++k) {
      const uint32_t c = s_wl[k];
      woff += (uint32_t)k < w ? c : 0u;
      total += c;
    }
    if (valid) {
      const int below = (int)s_ps[base + tid] + (int)cnt - 1;
      lmax = below > lmax ? below : lmax;
      int o = base + cur_n + (int)(woff + pre);
      for (int j = 0; j < 4; ++j)
        if (h[j] < kMidLeaf) {
          s_order[o] = (uint16_t)h[j];
          s_bfs[h[j]] = (uint16_t)o;
          s_ps[o] = (uint16_t)below;
          ++o;
        }
    }
    ++depth;
    __syncthreads();
    base += cur_n;
    cur_n = (int)total;
  }
  // 6. the 4-wide nodes
  for (int k = (int)tid; k < base; k += kTinyMax) {
    int ref[4];
    float box[4][6];
    const int cnt = wide_slots_dp(s_bin, s_dpc, s_dps, (int)s_order[k], ref, box, blas);
    write_wide_node(ref, box, cnt, s_bfs, out + k);
  }
  atomicMax(&s_maxstack, lmax);
  __syncthreads();
  if (tid == 0) {
    info[0] = (uint32_t)base;
    info[1] = (uint32_t)depth;
    info[2] = (uint32_t)s_maxstack;
  }
}

__global__ void k_tri_setup(const float* __restrict__ vtx, const uint32_t* __restrict__ idx,
                            uint32_t ntri, TriRec* __restrict__ tris, float* __restrict__ box) {
  uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= ntri) return;
  uint32_t i0 = idx ? idx[3 * p] : 3 * p, i1 = idx ? idx[3 * p + 1] : 3 * p + 1,
           i2 = idx ? idx[3 * p + 2] : 3 * p + 2;
  const float* a = vtx + (size_t)i0 * 6;
  const float* b = vtx + (size_t)i1 * 6;
  const float* c = vtx + (size_t)i2 * 6;
  TriRec t;
  for (int k = 0; k < 3; ++k) {
    t.v0[k] = a[k];
    t.e1[k] = b[k] - a[k];
    t.e2[k] = c[k] - a[k];
    // "+ 0.0f" turns -0 into +0: min/max of +-0 may return either sign, boxes must be canonical
    box[(size_t)p * 6 + k] = fminf(fminf(a[k], b[k]), c[k]) + 0.0f;
    box[(size_t)p * 6 + 3 + k] = fmaxf(fmaxf(a[k], b[k]), c[k]) + 0.0f;
  }
  t.prim = p;
  t.pad1 = t.pad2 = 0;
  tris[p] = t;
}

__global__ void k_tri_reorder(const TriRec* __restrict__ in, const uint32_t* __restrict__ sorted,
                              uint32_t n, TriRec* __restrict__ out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[sorted[i]];
}

__global__ void k_inst_boxes(const InstanceRec* __restrict__ inst, const float* __restrict__ bb,
                             uint32_t n, float* __restrict__ box) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* m = inst[i].o2w;
  const float* b = bb + (size_t)i * 6;
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int c = 0; c < 8; ++c) {
    V3 p = v3((c & 1) ? b[3] : b[0], (c & 2) ? b[4] : b[1], (c & 4) ? b[5] : b[2]);
    V3 w = xform_point(m, p);
    lo[0] = fminf(lo[0], w.x);
    lo[1] = fminf(lo[1], w.y);
    lo[2] = fminf(lo[2], w.z);
    hi[0] = fmaxf(hi[0], w.x);
    hi[1] = fmaxf(hi[1], w.y);
    hi[2] = fmaxf(hi[2], w.z);
  }
  for (int k = 0; k < 3; ++k) {
    box[(size_t)i * 6 + k] = lo[k] + 0.0f;  // canonical +0
    box[(size_t)i * 6 + 3 + k] = hi[k] + 0.0f;
  }
}

inline unsigned grid1(uint32_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

enum { kPathSmall = 0, kPathMid = 1, kPathMulti = 2, kPathTiny = 3 };

// Which schedule builds n primitives (measured crossovers). RT_BUILD_PATH=small|mid|multi
// in the environment forces one where it can hold n (A/B timing only; every schedule builds the
// bitwise-identical tree).
int build_path(uint32_t n) {
  const char* f = getenv("RT_BUILD_PATH");
  const bool small_ok = RT_FUSED_BUILD && n <= kFusedMax, mid_ok = RT_SAH_COLLAPSE && n >= 2 && n <= kMidMax;
  const bool tiny_ok = RT_SAH_COLLAPSE && n >= 2 && n <= kTinyMax;
  if (f) {
    if (!strcmp(f, "tiny") && tiny_ok) return kPathTiny;
    if (!strcmp(f, "small") && small_ok) return kPathSmall;
    if (!strcmp(f, "mid") && mid_ok) return kPathMid;
    if (!strcmp(f, "multi")) return kPathMulti;
  }
  if (RT_TINY_BUILD && tiny_ok && n <= (uint32_t)RT_TINY_MAX_N) return kPathTiny;
  if (RT_MID_BUILD && mid_ok && n >= (uint32_t)RT_MID_MIN_N) return kPathMid;
  if (small_ok && n <= (uint32_t)RT_FUSED_MAX_N) return kPathSmall;
  return kPathMulti;
}

struct DevBuf {
  void* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

#define RT_TRY(x)                         \
  do {                                    \
    hipError_t e_ = (x);                  \
    if (e_ != hipSuccess) return e_;      \
  } while (0)

}  // namespace

hipError_t lbvh_build(const float* d_primbox, uint32_t n, Bvh4Node* d_nodes, uint32_t* d_sorted,
                      bool leaf_ref_is_prim, uint32_t* node_count, uint32_t* depth, uint32_t* max_stack,
                      float bounds[6], float* build_ms, hipStream_t s, const TriRec* d_tri_in, TriRec* d_tri_out,
                      BuildArena* keep) {
  if (n == 0) return hipErrorInvalidValue;
  const uint32_t nblocks = (n + kRsTile - 1) / kRsTile;
  const uint32_t nbin = n > 1 ? n - 1 : 1;
  // all temporaries in ONE allocation (hipMalloc costs ~0.1 ms each; a hot-reload rebuild pays it)
  struct Part {
    size_t off, bytes;
  };
  size_t total = 0;
  auto part = [&](size_t bytes) {
    Part q{total, bytes};
    total += (bytes + 255) & ~(size_t)255;
    return q;
  };
  // stats and info first and adjacent: one readback copies both
  const Part p_stats = part(12 * sizeof(float)), p_info = part(32), p_keys0 = part((size_t)n * 4),
             p_keys1 = part((size_t)n * 4), p_vals1 = part((size_t)n * 4), p_hist = part((size_t)256 * nblocks * 4),
             p_ps = part((size_t)nbin * 4), p_bin = part((size_t)nbin * sizeof(BinNode)), p_la = part((size_t)nbin * 4),
             p_lb = part((size_t)nbin * 4), p_child = part((size_t)nbin * 8), p_pint = part((size_t)nbin * 4),
             p_pleaf = part((size_t)n * 4), p_nbox = part((size_t)nbin * 24), p_flags = part((size_t)nbin * 4),
             p_dpc = part(RT_SAH_COLLAPSE ? (size_t)nbin * sizeof(float4) : 0),
             p_dps = part(RT_SAH_COLLAPSE ? (size_t)nbin * 4 : 0),
             p_exp = part(RT_SAH_COLLAPSE ? (size_t)nbin * sizeof(Exp4) : 0),
             p_gslot = part((size_t)n * sizeof(MidSlot)), p_e16 = part((size_t)nbin * sizeof(uint2)),
             p_order = part((size_t)nbin * 2), p_bfs = part((size_t)nbin * 2),
             p_k64 = part((size_t)n * 8), p_sbox = part((size_t)n * 24);
  DevBuf arena;
  char* A = nullptr;
  if (keep) {  // the caller's scratch, kept between builds (no hipMalloc / hipFree on the way)
    if (keep->cap < total) {
      RT_TRY(hipStreamSynchronize(s));  // the previous build on s is the only user
      if (keep->p) RT_TRY(hipFree(keep->p));
      keep->p = nullptr;
      keep->cap = 0;
      RT_TRY(hipMalloc(&keep->p, total));
      keep->cap = total;
    }
    A = (char*)keep->p;
  } else {
    RT_TRY(hipMalloc(&arena.p, total));
    A = (char*)arena.p;
  }
  struct View {
    void* p;
  };
  auto at = [&](const Part& q) { return View{q.bytes ? (void*)(A + q.off) : nullptr}; };
  View stats = at(p_stats), keys0 = at(p_keys0), keys1 = at(p_keys1), vals1 = at(p_vals1), hist = at(p_hist),
       info = at(p_info), ps = at(p_ps), bin = at(p_bin), la = at(p_la), lb = at(p_lb), child = at(p_child),
       pint = at(p_pint), pleaf = at(p_pleaf), nbox = at(p_nbox), flags = at(p_flags), dpc = at(p_dpc),
       dps = at(p_dps), expd = at(p_exp), gslot = at(p_gslot), e16 = at(p_e16), order = at(p_order),
       bfsmap = at(p_bfs), k64 = at(p_k64), sbox = at(p_sbox);
  struct Events {  // destroyed on every return path
    hipEvent_t a = nullptr, b = nullptr;
    ~Events() {
      if (a) (void)hipEventDestroy(a);
      if (b) (void)hipEventDestroy(b);
    }
  } ev;
  hipEvent_t e0, e1;
  if (keep) {
    if (!keep->e0) RT_TRY(hipEventCreate(&keep->e0));
    if (!keep->e1) RT_TRY(hipEventCreate(&keep->e1));
    e0 = keep->e0;
    e1 = keep->e1;
  } else {
    RT_TRY(hipEventCreate(&ev.a));
    RT_TRY(hipEventCreate(&ev.b));
    e0 = ev.a;
    e1 = ev.b;
  }
  RT_TRY(hipEventRecord(e0, s));
  float* cb = (float*)stats.p;
  const int path = build_path(n);
  if (path == kPathTiny) {
    k_build_tiny<<<1, kTinyMax, 0, s>>>(d_primbox, n, leaf_ref_is_prim, d_sorted, cb, d_nodes, (uint32_t*)info.p,
                                        d_tri_in, d_tri_out);
    RT_TRY(hipGetLastError());
  } else if (path == kPathMid) {
    k_mid_rank<<<grid1(n, 64), 1024, 0, s>>>(d_primbox, n, cb, (uint64_t*)k64.p, (uint32_t*)keys0.p, d_sorted,
                                              (float*)sbox.p, (uint32_t*)dps.p, (uint32_t*)info.p, d_tri_in,
                                              d_tri_out);
    k_mid_tree<<<grid1(n, kMidBlock), kMidBlock, 0, s>>>(n, (const uint32_t*)keys0.p, d_sorted,
                                                          (const float*)sbox.p,
                                                          leaf_ref_is_prim, (BinNode*)bin.p, (float4*)dpc.p,
                                                          (uint32_t*)dps.p, (MidSlot*)gslot.p, (uint32_t*)info.p);
    k_mid_expand<<<grid1(nbin, 256), 256, 0, s>>>((int)nbin, (const BinNode*)bin.p, (const float4*)dpc.p,
                                                  (const uint32_t*)dps.p, (Exp4*)expd.p, (uint2*)e16.p,
                                                  !leaf_ref_is_prim);
    k_mid_collapse<<<1, 1024, 0, s>>>(n, (const uint32_t*)keys0.p, (const MidSlot*)gslot.p, (BinNode*)bin.p,
                                      (float4*)dpc.p, (uint32_t*)dps.p, (Exp4*)expd.p, (const uint2*)e16.p,
                                      (uint16_t*)order.p, (uint16_t*)bfsmap.p, (uint32_t*)info.p, !leaf_ref_is_prim);
    k_mid_write<<<grid1(nbin, 256), 256, 0, s>>>((const Exp4*)expd.p, (const uint16_t*)order.p,
                                                 (const uint16_t*)bfsmap.p, (const uint32_t*)info.p, d_nodes);
    RT_TRY(hipGetLastError());
  } else if (path == kPathSmall) {
    k_build_small<<<1, kFusedThreads, 0, s>>>(d_primbox, n, leaf_ref_is_prim, d_sorted, cb, (int*)pleaf.p,
                                              (float*)nbox.p, (float4*)dpc.p, (uint32_t*)dps.p, (BinNode*)bin.p,
                                              d_nodes, (uint32_t*)info.p, d_tri_in, d_tri_out);
    RT_TRY(hipGetLastError());
  } else {
  k_bounds<<<1, 1024, 0, s>>>(d_primbox, n, cb);
  RT_TRY(hipGetLastError());
  uint32_t* ka = (uint32_t*)keys0.p;
  uint32_t* va = d_sorted;  // values ping-pong between d_sorted and vals1; 4 passes end in d_sorted
  uint32_t* kb = (uint32_t*)keys1.p;
  uint32_t* vb = (uint32_t*)vals1.p;
  k_morton<<<grid1(n, 256), 256, 0, s>>>(d_primbox, n, cb, ka, va);
  RT_TRY(hipGetLastError());
  for (int pass = 0; pass < 4; ++pass) {
    int shift = pass * 8;
    k_rs_hist<<<nblocks, kRsThreads, 0, s>>>(ka, n, shift, (uint32_t*)hist.p, nblocks);
    k_rs_scan<<<1, 1024, 0, s>>>((uint32_t*)hist.p, 256 * nblocks);
    k_rs_scatter<<<nblocks, kRsThreads, 0, s>>>(ka, va, kb, vb, n, shift, (uint32_t*)hist.p, nblocks);
    RT_TRY(hipGetLastError());
    std::swap(ka, kb);
    std::swap(va, vb);
  }
  // after 4 swaps: va == d_sorted, ka == keys0 (sorted keys)
  BinNode* d_bin = (BinNode*)bin.p;
  if (n == 1) {
    k_single<<<1, 1, 0, s>>>(d_primbox, leaf_ref_is_prim, d_bin);
    RT_TRY(hipGetLastError());
  } else {
    RT_TRY(hipMemsetAsync(flags.p, 0, (size_t)(n - 1) * 4, s));
    k_karras<<<grid1(n - 1, 256), 256, 0, s>>>(ka, (int)n, (int*)child.p, (int*)pint.p, (int*)pleaf.p);
    k_refit<<<grid1(n, 256), 256, 0, s>>>((int)n, (int*)pleaf.p, (int*)pint.p, (int*)child.p, d_primbox,
                                          d_sorted, (float*)nbox.p, (uint32_t*)flags.p, (float4*)dpc.p,
                                          (uint32_t*)dps.p);
    k_pack<<<grid1(n - 1, 256), 256, 0, s>>>((int)n, (int*)child.p, (float*)nbox.p, d_primbox, d_sorted,
                                             leaf_ref_is_prim, d_bin);
    RT_TRY(hipGetLastError());
  }
  if (RT_SAH_COLLAPSE) {
    k_dp_expand<<<grid1(nbin, 256), 256, 0, s>>>((int)nbin, d_bin, (const float4*)dpc.p, (const uint32_t*)dps.p,
                                                 (Exp4*)expd.p, !leaf_ref_is_prim);
    RT_TRY(hipGetLastError());
  }
  k_collapse<<<1, 1024, 0, s>>>(d_bin, (const Exp4*)expd.p, d_nodes, (int*)la.p, (int*)lb.p, (int*)ps.p,
                                (uint32_t*)info.p, !leaf_ref_is_prim);
  RT_TRY(hipGetLastError());
  if (d_tri_in) {
    k_tri_reorder<<<grid1(n, 256), 256, 0, s>>>(d_tri_in, d_sorted, n, d_tri_out);
    RT_TRY(hipGetLastError());
  }
  }
  RT_TRY(hipEventRecord(e1, s));
  float hb[12];
  uint32_t hinfo[3];
  const size_t info_off = p_info.off - p_stats.off;  // 256: the parts are adjacent
  if (keep) {  // one copy of both into the arena's pinned buffer (a pageable destination is staged by the runtime)
    if (!keep->host) RT_TRY(hipHostMalloc(&keep->host, info_off + 32, hipHostMallocDefault));
    RT_TRY(hipMemcpyAsync(keep->host, cb, info_off + 12, hipMemcpyDeviceToHost, s));
    RT_TRY(hipStreamSynchronize(s));
    std::memcpy(hb, keep->host, sizeof(hb));
    std::memcpy(hinfo, (const char*)keep->host + info_off, sizeof(hinfo));
  } else {
    RT_TRY(hipMemcpyAsync(hb, cb, sizeof(hb), hipMemcpyDeviceToHost, s));
    RT_TRY(hipMemcpyAsync(hinfo, info.p, 12, hipMemcpyDeviceToHost, s));
    RT_TRY(hipStreamSynchronize(s));
  }
  for (int k = 0; k < 6; ++k) bounds[k] = hb[6 + k];
  *node_count = hinfo[0];
  *depth = hinfo[1];
  *max_stack = hinfo[2];
  float ms = 0.0f;
  RT_TRY(hipEventElapsedTime(&ms, e0, e1));
  if (build_ms) *build_ms = ms;
  return hipSuccess;
}

namespace {
__global__ void k_pool_rebase(const Bvh4Node* __restrict__ src, uint32_t n, uint32_t node_base, int64_t tri_base,
                              Bvh4Node* __restrict__ dst) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Bvh4Node nd = src[i];
  for (int k = 0; k < 4; ++k) {
    const int32_t c = nd.child[k];
    if (c == kEmptyChild) continue;
    if (c >= 0) nd.child[k] = c + (int32_t)node_base;
    else if (tri_base >= 0) nd.child[k] = ~(int32_t)((int64_t)(~c) + tri_base);
  }
  if (nd.inner_mask) nd.first_inner += (int32_t)node_base;
  nd.entry_base = ((uint32_t)nd.first_inner << 8) | (nd.inner_mask << 4);
  dst[i] = nd;
}
}  // namespace

hipError_t pool_rebase(const Bvh4Node* src, uint32_t n, uint32_t node_base, int64_t tri_base, Bvh4Node* dst,
                       hipStream_t s) {
  k_pool_rebase<<<grid1(n, 256), 256, 0, s>>>(src, n, node_base, tri_base, dst);
  return hipGetLastError();
}

hipError_t blas_prepare(const float* d_vtx, const uint32_t* d_idx, uint32_t ntri, TriRec* d_tris,
                        float* d_primbox, hipStream_t s) {
  k_tri_setup<<<grid1(ntri, 256), 256, 0, s>>>(d_vtx, d_idx, ntri, d_tris, d_primbox);
  return hipGetLastError();
}

hipError_t blas_reorder(const TriRec* d_in, const uint32_t* d_sorted, uint32_t n, TriRec* d_out,
                        hipStream_t s) {
  k_tri_reorder<<<grid1(n, 256), 256, 0, s>>>(d_in, d_sorted, n, d_out);
  return hipGetLastError();
}

hipError_t tlas_prepare(const InstanceRec* d_inst, const float* d_blas_bounds, uint32_t n,
                        float* d_primbox, hipStream_t s) {
  k_inst_boxes<<<grid1(n, 64), 64, 0, s>>>(d_inst, d_blas_bounds, n, d_primbox);
  return hipGetLastError();
}

}  // namespace rt
