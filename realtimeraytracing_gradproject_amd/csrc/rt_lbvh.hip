// rt_lbvh.hip — on-device LBVH build for BLAS and TLAS on gfx950.
//
// Replaces the driver acceleration-structure builds behind
//   BottomLevelASGenerator::Generate  nv_helpers_dx12/BottomLevelASGenerator.cpp:177-245 (build :234)
//   TopLevelASGenerator::Generate     nv_helpers_dx12/TopLevelASGenerator.cpp:148-249 (build :239)
//
// Pipeline (all deterministic, so oracle/rt_oracle.c rebuilds the bit-identical tree):
//   1. centroid bounds      one 1024-thread workgroup, LDS min/max reduction (exact)
//   2. Morton codes         30-bit (10 bits/axis) of box centroids
//   3. LSD radix sort       4 passes x 8 bits; per pass: block digit histogram (LDS atomics),
//                           exclusive scan, stable scatter with wave64 ballot match + popcount
//                           ranks (keys tie-break on primitive index: stable)
//   4. Karras hierarchy     Karras 2012 over key64 = morton << 32 | leaf position
//   5. bottom-up refit      one thread per leaf, agent-scope release/acquire arrival counters
//   6. pack                 64-B child-pair nodes (both child boxes per node)
#include <hip/hip_runtime.h>

#include <vector>

#include "rt_internal.hpp"

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
__device__ __forceinline__ void sah_dp(int node, const float* bb, int c0, int c1, float4* __restrict__ dpc,
                                       uint32_t* __restrict__ dps) {
  const float4 zero = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  const float4 l = c0 >= 0 ? dpc[c0] : zero, r = c1 >= 0 ? dpc[c1] : zero;
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
  dpc[node] = make_float4(C[1], C[2], C[3], C[4]);
  dps[node] = S;
}

__global__ void k_refit(int n, const int* __restrict__ parent_leaf, const int* __restrict__ parent_int,
                        const int* __restrict__ child, const float* __restrict__ primbox,
                        const uint32_t* __restrict__ sorted, float* nbox, uint32_t* flags,
                        float4* __restrict__ dpc, uint32_t* __restrict__ dps) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int node = parent_leaf[i];
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

// The DP expansion of every binary node, in parallel (only wide-node roots are read): k_collapse
// then takes one record per node instead of walking dependent loads level by level.
struct alignas(128) Exp4 {
  int ref[4];
  float box[4][6];
  int cnt, pad[3];
};

__global__ void k_dp_expand(int nbin, const BinNode* __restrict__ bin, const float4* __restrict__ dpc,
                            const uint32_t* __restrict__ dps, Exp4* __restrict__ exp) {
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
  e.pad[0] = e.pad[1] = e.pad[2] = 0;
  exp[i] = e;
}

__global__ __launch_bounds__(1024) void k_collapse(const BinNode* __restrict__ bin, const Exp4* __restrict__ exp,
                                                   Bvh4Node* __restrict__ out,
                                                   int* la, int* lb, int* ps, uint32_t* __restrict__ info) {
  __shared__ int scan[1024];
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
        }
      }
      int m = 0;
      for (int j = 0; j < cnt; ++j) m += ref[j] >= 0;
      scan[tid] = m;
      __syncthreads();
      for (int off = 1; off < 1024; off <<= 1) {
        const int add = tid >= off ? scan[tid - off] : 0;
        __syncthreads();
        scan[tid] += add;
        __syncthreads();
      }
      const int excl = scan[tid] - m;
      const int chunk_total = scan[1023];
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
                      float bounds[6], float* build_ms, hipStream_t s) {
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
  const Part p_stats = part(12 * sizeof(float)), p_keys0 = part((size_t)n * 4), p_keys1 = part((size_t)n * 4),
             p_vals1 = part((size_t)n * 4), p_hist = part((size_t)256 * nblocks * 4), p_info = part(12),
             p_ps = part((size_t)nbin * 4), p_bin = part((size_t)nbin * sizeof(BinNode)), p_la = part((size_t)nbin * 4),
             p_lb = part((size_t)nbin * 4), p_child = part((size_t)nbin * 8), p_pint = part((size_t)nbin * 4),
             p_pleaf = part((size_t)n * 4), p_nbox = part((size_t)nbin * 24), p_flags = part((size_t)nbin * 4),
             p_dpc = part(RT_SAH_COLLAPSE ? (size_t)nbin * sizeof(float4) : 0),
             p_dps = part(RT_SAH_COLLAPSE ? (size_t)nbin * 4 : 0),
             p_exp = part(RT_SAH_COLLAPSE ? (size_t)nbin * sizeof(Exp4) : 0);
  DevBuf arena;
  RT_TRY(hipMalloc(&arena.p, total));
  char* A = (char*)arena.p;
  struct View {
    void* p;
  };
  auto at = [&](const Part& q) { return View{q.bytes ? (void*)(A + q.off) : nullptr}; };
  View stats = at(p_stats), keys0 = at(p_keys0), keys1 = at(p_keys1), vals1 = at(p_vals1), hist = at(p_hist),
       info = at(p_info), ps = at(p_ps), bin = at(p_bin), la = at(p_la), lb = at(p_lb), child = at(p_child),
       pint = at(p_pint), pleaf = at(p_pleaf), nbox = at(p_nbox), flags = at(p_flags), dpc = at(p_dpc),
       dps = at(p_dps), expd = at(p_exp);
  hipEvent_t e0, e1;
  RT_TRY(hipEventCreate(&e0));
  RT_TRY(hipEventCreate(&e1));
  RT_TRY(hipEventRecord(e0, s));
  float* cb = (float*)stats.p;
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
                                                 (Exp4*)expd.p);
    RT_TRY(hipGetLastError());
  }
  k_collapse<<<1, 1024, 0, s>>>(d_bin, (const Exp4*)expd.p, d_nodes, (int*)la.p, (int*)lb.p, (int*)ps.p,
                                (uint32_t*)info.p);
  RT_TRY(hipGetLastError());
  RT_TRY(hipEventRecord(e1, s));
  float hb[12];
  uint32_t hinfo[3];
  RT_TRY(hipMemcpyAsync(hb, cb, sizeof(hb), hipMemcpyDeviceToHost, s));
  RT_TRY(hipMemcpyAsync(hinfo, info.p, 12, hipMemcpyDeviceToHost, s));
  RT_TRY(hipStreamSynchronize(s));
  for (int k = 0; k < 6; ++k) bounds[k] = hb[6 + k];
  *node_count = hinfo[0];
  *depth = hinfo[1];
  *max_stack = hinfo[2];
  float ms = 0.0f;
  RT_TRY(hipEventElapsedTime(&ms, e0, e1));
  if (build_ms) *build_ms = ms;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
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
