// rt_trace.hip — the trace megakernel: RayGen -> TLAS/BLAS traversal + Moller-Trumbore ->
// ClosestHit / PlaneClosestHit (+ shadow rays) / Miss -> RGBA8, in one launch on gfx950.
//
// Replaces DispatchRays (D3D12HelloTriangle.cpp:558-592) and the DXR programs:
//   RayGen            shaders/RayGen.hlsl:28-43
//   CastDefaultRay    shaders/Common.hlsl:44-56   (TMin 0, TMax 1e5, no culling)
//   CastShadowRay     shaders/Common.hlsl:71-82   (TMin 0.01, TMax 1e5, any hit terminates)
//   ClosestHit        shaders/Hit.hlsl:183-204    (+ :67-174 normal, Lambert, PBR)
//   PlaneClosestHit   shaders/Hit.hlsl:207-241
//   Miss              shaders/Miss.hlsl:3-10
//   ShadowClosestHit / ShadowMiss  shaders/ShadowRay.hlsl:10-20
// SBT dispatch (D3D12HelloTriangle.cpp:1064-1080) becomes a switch on the instance hit group.
//
// Execution model: one lane = one pixel, a wave64 = an 8x8 pixel tile, a 256-thread workgroup =
// 16x16 pixels. 4-wide BVH nodes (128 B, one cache line) from the scene pool: one node fetch
// tests four children, visited nearest first. Per-lane traversal stack in LDS laid out
// [entry][lane] (bank = lane: conflict free) with an HBM overflow for deep paths.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <utility>
#include <vector>

#include "../../include/rt_api.h"
#include "rt_internal.hpp"

// v_writelane_b32 (the LLVM intrinsic; this clang has no builtin for it): writes the uniform x
// into lane l of v, whatever EXEC holds.
__device__ int amdgcn_writelane(int x, int l, int v) __asm("llvm.amdgcn.writelane.i32");

namespace rt {
namespace {

constexpr int kBlock = 256;
constexpr float kPi = 3.14159265359f;  // Common.hlsl:1

struct Counters {
  uint32_t primary = 0, shadow = 0, aabb = 0, tri = 0, inst = 0, overflow = 0, refl = 0;
  // record fetches (RT_STAT_*_FETCHES): per lane in the per-lane schedule; in the packet schedule
  // wave-uniform (every lane holds the wave's count, flushed once per wave)
  uint32_t nfetch = 0, tfetch = 0, ifetch = 0;
  // record fetches of per-lane subtree walks inside the packet schedule (lane_subtree): per lane, summed
  // over the wave at the flush and added to the node / triangle fetch slots
  uint32_t lnfetch = 0, ltfetch = 0;
};

struct HitRec {
  float t, u, v;
  uint32_t inst;  // instance index (== InstanceID() of the reference list)
  uint32_t prim;  // PrimitiveIndex()
};

__device__ __forceinline__ V3 ld3(const float* p) { return v3(p[0], p[1], p[2]); }

// Scene data is read through explicit global (address space 1) pointers: pointers loaded from
// memory (instance records) would otherwise become flat accesses, which wait on both vmcnt and
// lgkmcnt and serialise the node fetch against LDS stack traffic.
#define RT_GLOBAL __attribute__((address_space(1)))
typedef float f4v __attribute__((ext_vector_type(4)));
typedef int i4v __attribute__((ext_vector_type(4)));
typedef int i8v __attribute__((ext_vector_type(8)));
typedef float f8v __attribute__((ext_vector_type(8)));
#ifndef RT_REF0_WAVES
#define RT_REF0_WAVES 6  // the reflectivity-0 REF kernel (MODE 3, one sample): 73 VGPRs, no spills (7 waves: 2
                         // spilled VGPRs, the same frame time)
#endif
#ifndef RT_REF_NOREFL
#define RT_REF_NOREFL 1  // RT_SHADE_REF with reflectivity 0: the kernel specialised without reflection rays
#endif
#ifndef RT_PACKET_OCT
#define RT_PACKET_OCT 1  // uniform-octant BLAS walks load near/far planes directly (no min/max pairs)
#endif
template <typename T>
__device__ __forceinline__ const RT_GLOBAL T* gp(const T* p) {
  return (const RT_GLOBAL T*)p;
}

// Per-lane stack: entries [0, lds_cap) in LDS ([entry][lane], bank = lane), deeper entries in
// the HBM overflow area ([entry - lds_cap][lane]), touched only by paths deeper than lds_cap.
// The capacity is the exact worst case of the scene's trees, so nothing is ever dropped.
struct LaneStack {
  int* lds;                 // s_stack + threadIdx.x
  RT_GLOBAL int* ovf;       // overflow base + global lane (null when stack_cap <= lds_cap)
  uint32_t pitch;           // lanes of the launch
  int lds_cap, cap;
  __device__ __forceinline__ void put(int slot, int v) const {
    if (slot < lds_cap) lds[slot * kBlock] = v;
    else if (slot < cap) ovf[(size_t)(slot - lds_cap) * pitch] = v;
  }
  __device__ __forceinline__ int get(int slot) const {
    int v;
    if (slot < lds_cap) v = lds[slot * kBlock];
    else v = ovf[(size_t)(slot - lds_cap) * pitch];
    return v;
  }
};

__device__ __forceinline__ LaneStack lane_stack(const SceneView& sc, int* s_stack, uint32_t global_lane) {
  LaneStack st;
  st.lds = s_stack + threadIdx.x;
  st.ovf = sc.ovf ? (RT_GLOBAL int*)sc.ovf + global_lane : nullptr;
  st.pitch = sc.ovf_lanes;
  st.lds_cap = sc.lds_cap;
  st.cap = sc.stack_cap;
  return st;
}

// Pool loads: uniform (SGPR) base + 32-bit per-lane byte offset, the global_load saddr form.
__device__ __forceinline__ f4v ldf4(const RT_GLOBAL char* base, uint32_t off) {
  return *reinterpret_cast<const RT_GLOBAL f4v*>(base + off);
}
__device__ __forceinline__ i4v ldi4(const RT_GLOBAL char* base, uint32_t off) {
  return *reinterpret_cast<const RT_GLOBAL i4v*>(base + off);
}

// Byte offsets of the near planes inside a Bvh4Node for the ray's octant (the far plane of an
// axis is the near one ^ 16): lox 0, hix 16, loy 32, hiy 48, loz 64, hiz 80.
struct Octant {
  uint32_t x, y, z;
};
__device__ __forceinline__ Octant octant(V3 invd) {
  Octant q;
  q.x = invd.x < 0.0f ? 16u : 0u;
  q.y = invd.y < 0.0f ? 48u : 32u;
  q.z = invd.z < 0.0f ? 80u : 64u;
  return q;
}

// Two-level stack traversal over the scene pool. ANY_HIT: first accepted hit terminates (shadow
// rays). Closest hit keeps the lexicographic minimum of (t, instance, primitive): independent of
// traversal order. Children are visited nearest first (sort4); the oracle mirrors the order, so
// the box/triangle test counters match it exactly. Entering an instance pushes a sentinel and
// moves to the BLAS root in the pool; popping the sentinel restores the world-space ray.
template <bool ANY_HIT, bool STATS, bool CULL = false>
__device__ bool trace(const SceneView& sc, V3 o, V3 d, float tmin, float tmax, HitRec& hit,
                      const LaneStack& stk, Counters& cnt) {
  const V3 winvd = v3(safe_inv(d.x), safe_inv(d.y), safe_inv(d.z));
  const V3 wnoinv = neg(mul(o, winvd));
  const Octant woct = octant(winvd);
  V3 ro = o, rd = d, rinvd = winvd, rnoinv = wnoinv;
  Octant oct = woct;
  const RT_GLOBAL char* pn = (const RT_GLOBAL char*)sc.pool_nodes;
  const RT_GLOBAL char* pt = (const RT_GLOBAL char*)sc.pool_tris;
  uint32_t cur = 0;
  float face = 0.0f;  // CULL: +1 / -1 (mirroring instance) for the current BLAS
  bool in_blas = false;
  bool found = false;
  const int cap = stk.cap;
  int sp = 0;
  int ref = sc.tlas_root;
  hit.t = tmax;
  hit.inst = 0xffffffffu;
  hit.prim = 0xffffffffu;
  hit.u = hit.v = 0.0f;
  while (true) {
    if (ref >= 0) {
      const uint32_t off = (uint32_t)ref << 7;
      const f4v a0 = ldf4(pn, off + oct.x), a1 = ldf4(pn, off + (oct.x ^ 16u));
      const f4v a2 = ldf4(pn, off + oct.y), a3 = ldf4(pn, off + (oct.y ^ 16u));
      const f4v a4 = ldf4(pn, off + oct.z), a5 = ldf4(pn, off + (oct.z ^ 16u));
      const i4v ch = ldi4(pn, off + 96u);
      const float nx[4] = {a0.x, a0.y, a0.z, a0.w}, fx[4] = {a1.x, a1.y, a1.z, a1.w};
      const float ny[4] = {a2.x, a2.y, a2.z, a2.w}, fy[4] = {a3.x, a3.y, a3.z, a3.w};
      const float nz[4] = {a4.x, a4.y, a4.z, a4.w}, fz[4] = {a5.x, a5.y, a5.z, a5.w};
      int32_t r[4] = {ch.x, ch.y, ch.z, ch.w};
      float tn[4];
      slab4_octant(nx, fx, ny, fy, nz, fz, r, rinvd, rnoinv, tmin, hit.t, tn);
      if (STATS) ++cnt.nfetch;
      if (STATS)
        cnt.aabb += (uint32_t)(r[0] != kEmptyChild) + (uint32_t)(r[1] != kEmptyChild) +
                    (uint32_t)(r[2] != kEmptyChild) + (uint32_t)(r[3] != kEmptyChild);
      sort4(tn, r);
      if (tn[0] != __builtin_inff()) {
#pragma unroll
        for (int k = 3; k >= 1; --k) {
          const bool h = tn[k] != __builtin_inff();
          if (h) {
            if (sp < cap) {
              stk.put(sp, r[k]);
              ++sp;
            } else if (STATS) {
              ++cnt.overflow;
            }
          }
        }
        ref = r[0];
        continue;
      }
    } else if (!in_blas) {
      cur = (uint32_t)(~ref);
      const RT_GLOBAL InstanceRec* ir = gp(sc.inst) + cur;
      if (STATS) ++cnt.inst;
      if (STATS) ++cnt.ifetch;
      if (sp < cap) {
        stk.put(sp, kStackSentinel);
        ++sp;
        float m[12];
        for (int k = 0; k < 12; ++k) m[k] = ir->w2o[k];
        const uint32_t tr = ir->translate;
        ro = inst_point(m, tr, o);
        rd = inst_dir(m, tr, d);
        rinvd = tr ? winvd : v3(safe_inv(rd.x), safe_inv(rd.y), safe_inv(rd.z));
        rnoinv = neg(mul(ro, rinvd));
        oct = octant(rinvd);
        if (CULL) face = (ir->flip ? -1.0f : 1.0f) * sc.cull_sense;
        in_blas = true;
        ref = (int)ir->pool_root;
        continue;
      }
      if (STATS) ++cnt.overflow;  // no room for the way back: skip this instance
    } else {
      const uint32_t toff = (uint32_t)(~ref) * (uint32_t)sizeof(TriRec);
      const f4v a = ldf4(pt, toff), b = ldf4(pt, toff + 16u), c = ldf4(pt, toff + 32u);
      if (STATS) ++cnt.tri;
      if (STATS) ++cnt.tfetch;
      float t, u, v;
      if (moller_trumbore(ro, rd, v3(a.x, a.y, a.z), v3(b.x, b.y, b.z), v3(c.x, c.y, c.z), face, t, u, v) &&
          t >= tmin) {
        const uint32_t prim = __float_as_uint(a.w);
        const bool better =
            t < hit.t || (t == hit.t && (cur < hit.inst || (cur == hit.inst && prim < hit.prim)));
        if (better) {
          hit.t = t;
          hit.u = u;
          hit.v = v;
          hit.inst = cur;
          hit.prim = prim;
          found = true;
          if (ANY_HIT) return true;
        }
      }
    }
    // pop
    while (true) {
      if (sp == 0) return found;
      --sp;
      ref = stk.get(sp);
      if (ref != kStackSentinel) break;
      in_blas = false;
      ro = o;
      rd = d;
      rinvd = winvd;
      rnoinv = wnoinv;
      oct = woct;
    }
  }
}

// ------------------------------------------------------------------------------------------
// Wave-packet traversal: the rays of a wave walk ONE path through the trees together. A packet
// is 64 x R rays: each lane carries R rays (R = 1: an 8x8 pixel tile per wave; R = 2: 8x16).
// The current node / triangle / instance is wave-uniform, so it is fetched with scalar loads
// into SGPRs (one fetch per wave instead of one per lane) and every lane tests its own rays
// against it; a child is entered when any live ray accepts it (ballots). The traversal stack is
// wave-uniform and lives in the 64 lanes of one VGPR (v_writelane / v_readlane): no LDS and no
// per-lane stack traffic. Children are ordered by the entry distance of the lead ray (the first
// live ray in slot order r * 64 + lane). All per-node decisions are scalar (SALU) work shared by
// the packet's 64 x R rays: R > 1 spends more VALU per node to amortise the SALU further.
// Results are those of the per-ray traversal: the closest hit is the lexicographic minimum of
// (t, instance, primitive) over every triangle a ray reaches, and every triangle whose root
// path the ray's slab tests accept is visited, whatever the order; a ray dragged into a leaf by
// other lanes takes no hit there unless its own test accepted the triangle's box (packet_tri).
// ------------------------------------------------------------------------------------------
#define RT_CONST __attribute__((address_space(4)))

constexpr int kPacketStack = 64;  // wave-uniform stack entries: one VGPR, entry i in lane i

struct WaveStack {
  int v = 0;
  __device__ __forceinline__ void put(int slot, int x) { v = amdgcn_writelane(x, slot, v); }
  __device__ __forceinline__ int get(int slot) const { return __builtin_amdgcn_readlane(v, slot); }
};

__device__ __forceinline__ uint64_t wave_ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

__device__ __forceinline__ f4v cld4(const RT_CONST char* p) { return *(const RT_CONST f4v*)p; }

// key where bit k of the uniform entered set m is set, else all ones (v_bfe_i32 + v_bfi_b32 on the
// SGPR m: no scalar instruction to invert m first)
__device__ __forceinline__ uint32_t key_if_entered(uint32_t key, uint32_t m, int k) {
  uint32_t r, t;
  asm("v_bfe_i32 %0, %2, %3, 1\n\t"
      "v_bfi_b32 %1, %0, %4, -1"
      : "=&v"(t), "=v"(r)
      : "s"(m), "i"(k), "v"(key));
  return r;
}

// Pushes entry_base | P with P = ent & ~nearest when P != 0: the write goes to lane sp, and sp
// advances by SCC (= P != 0): four scalar instructions and, when P != 0, one v_writelane (its lane
// select goes through m0, placed by the compiler: gfx9 VOP3 reads one SGPR per instruction, so value
// and lane cannot both be SGPRs).
__device__ __forceinline__ int push_entry(int stk, int& sp, uint32_t entry_base, uint32_t ent, uint32_t nearest) {
  uint32_t p, e, lane;
  asm volatile(
      "s_andn2_b32 %0, %4, %5\n\t"
      "s_cselect_b32 %3, %1, 63\n\t"
      "s_addc_u32 %1, %1, 0\n\t"
      "s_or_b32 %2, %6, %0"
      : "=&s"(p), "+s"(sp), "=&s"(e), "=&s"(lane)
      : "s"(ent), "s"(nearest), "s"(entry_base)
      : "scc");
  // nothing pending: a uniform branch around the write (round 6, with the pop's below: −0.1 … −1.1 % per config)
  if (p) stk = amdgcn_writelane((int)e, (int)lane, stk);
  return stk;
}

// Pops the packet walk's top BLAS entry (sp > base): returns its lowest pending child and keeps
// the entry, minus that slot, while slots remain. BLAS nodes hold their internal children in the
// lowest slots (inner_first in rt_lbvh.hip), so the child in slot k is first_inner + k (the lowest
// set bit of e is the lowest pending slot: the pending bits are the low four, never all zero).
// e & (e - 1) clears it.
__device__ __forceinline__ int pop_entry(int& stk, int& sp) {
  const int top = sp - 1;
  const uint32_t e = (uint32_t)__builtin_amdgcn_readlane(stk, top);
  uint32_t ref, rest, lane, t0, t1;
  asm volatile(
      "s_ff1_i32_b32 %3, %6\n\t"
      "s_lshr_b32 %0, %6, 8\n\t"
      "s_add_u32 %0, %0, %3\n\t"
      "s_add_u32 %4, %6, -1\n\t"
      "s_and_b32 %1, %6, %4\n\t"
      "s_and_b32 %4, %1, 15\n\t"
      "s_cselect_b32 %2, %7, 63\n\t"
      "s_cselect_b32 %5, %5, %7"
      : "=&s"(ref), "=&s"(rest), "=&s"(lane), "=&s"(t0), "=&s"(t1), "+s"(sp)
      : "s"(e), "s"(top)
      : "scc");
  if (t1) stk = amdgcn_writelane((int)rest, (int)lane, stk);  // the entry is done: nothing to write back
  return (int)ref;
}

// Bit k set iff the uniform 64-bit mask m[k] is nonzero: s_cmp_lg_u64 sets SCC and
// s_addc_u32 acc, acc, acc shifts it in (children 3..0), two scalar instructions per child.
__device__ __forceinline__ uint32_t nonzero_mask4(const uint64_t (&m)[4]) {
  uint32_t r;
  asm("s_cmp_lg_u64 %1, 0\n\t"
      "s_addc_u32 %0, 0, 0\n\t"
      "s_cmp_lg_u64 %2, 0\n\t"
      "s_addc_u32 %0, %0, %0\n\t"
      "s_cmp_lg_u64 %3, 0\n\t"
      "s_addc_u32 %0, %0, %0\n\t"
      "s_cmp_lg_u64 %4, 0\n\t"
      "s_addc_u32 %0, %0, %0"
      : "=&s"(r)
      : "s"(m[3]), "s"(m[2]), "s"(m[1]), "s"(m[0])
      : "scc");
  return r;
}


// Live rays of the packet: one ballot mask per ray slot r, and the lead ray (lowest r, then
// lowest lane).
// A ray is live while its t is not -inf: rays that are not alive start at -inf, and an any-hit ray
// that accepts a hit goes to -inf (no per-lane flag to maintain).
__device__ __forceinline__ bool ray_live(const HitRec& h) { return __float_as_uint(h.t) != 0xff800000u; }

template <int R>
struct PacketLive {
  uint64_t mask[R];
  uint32_t lead_r, lead_l;
  __device__ __forceinline__ bool update(const HitRec* hit) {  // false when no ray is live
    bool any = false;
    lead_r = 0;
    lead_l = 0;
#pragma unroll
    for (int r = R - 1; r >= 0; --r) {
      mask[r] = wave_ballot(ray_live(hit[r]));
      if (mask[r]) {
        any = true;
        lead_r = (uint32_t)r;
        lead_l = (uint32_t)__builtin_ctzll(mask[r]);
      }
    }
    return any;
  }
};

// Per-wave ray state of one traversal level (world rays in the TLAS, object rays in a BLAS).
template <int R>
struct PacketRay {
  V3 o[R], d[R], invd[R], noinv[R];
};

// Triangle leaf for every live ray (uniform triangle, scalar loads). ANY_HIT: a ray that accepts
// a hit leaves the packet. Branch-free: selects instead of exec-mask regions.
// own[r]: the lanes whose ray r accepted this triangle's slot box (the node's ballot for the slot). Only they may
// take a hit: a ray the packet drags into a leaf its own slab test rejected would otherwise see Moller-Trumbore's
// float32 false positives — a grazing ray passing just outside a triangle corner (float64 barycentrics ~-1e-4, a
// point outside the triangle's box) — which the per-ray walk never tests. With the mask a ray's accepted set is the
// per-ray walk's: a hit needs the triangle's own box, which implies every ancestor box (their planes enclose it and
// the fma is monotone in the plane), so the image does not depend on the schedule. One s_and_b64 per test.
template <bool ANY_HIT, bool STATS, int R>
__device__ __forceinline__ void packet_tri(const RT_CONST TriRec* tpool, int ref, const PacketRay<R>& ry,
                                           float tmin, uint32_t cur, float face, PacketLive<R>& pl, HitRec* hit,
                                           const uint64_t* own, Counters& cnt) {
  // 32-bit byte offsets (pools are < 2 GiB): the scalar load takes them as its SGPR offset
  const RT_CONST char* tq = (const RT_CONST char*)tpool + (uint32_t)(~ref) * 48u;
  const f8v tab = *(const RT_CONST f8v*)tq;  // one s_load_dwordx8 + one x4 for the 48-B record
  const f4v tc = *(const RT_CONST f4v*)(tq + 32);
  const f4v ta = {tab[0], tab[1], tab[2], tab[3]}, tb = {tab[4], tab[5], tab[6], tab[7]};
  const uint32_t prim = __float_as_uint(ta.w);
  if (STATS) ++cnt.tfetch;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (STATS && ray_live(hit[r])) ++cnt.tri;
    float t, u, v;
    const bool ok = moller_trumbore_flat(ry.o[r], ry.d[r], v3(ta.x, ta.y, ta.z), v3(tb.x, tb.y, tb.z),
                                         v3(tc.x, tc.y, tc.z), face, t, u, v);
    HitRec& h = hit[r];
    // bitwise & / | (no short-circuit): no exec-mask branches around the compares (-2 %)
    // a ray that is not live has t = -inf and takes nothing; a live any-hit ray still holds
    // {tmax, ~0, ~0}, for which the (t, instance, primitive) order reduces to t <= tmax
    // (instance, primitive) order as ONE unsigned 64-bit compare (v_cmp_lt_u64; the uniform side in an SGPR pair)
    const bool id_less = (((uint64_t)cur << 32) | prim) < (((uint64_t)h.inst << 32) | h.prim);
    const bool better = ANY_HIT ? (t <= h.t) : (t < h.t) | ((t == h.t) & id_less);
    const bool take = ok & (t >= tmin) & better & __builtin_amdgcn_inverse_ballot_w64(own[r]);
    // an any-hit ray that accepts leaves the packet with t = -inf: every later slab test rejects it
    h.t = take ? (ANY_HIT ? -__builtin_inff() : t) : h.t;
    h.u = take ? u : h.u;
    h.v = take ? v : h.v;
    h.inst = take ? cur : h.inst;
    h.prim = take ? prim : h.prim;
  }
}

// Slab tests of the 4 children of one node for every live ray: hm[r][k] = the live lanes whose
// ray r accepts child k, vkey[r][k] = |entry distance| where accepted, else +inf. Returns the
// entered set (children some live ray accepts). Unused slots hold lo = hi = +inf boxes that every
// ray rejects: no validity mask.
// Byte offsets, inside a node, of the near and far plane rows of each axis for one ray octant.
struct NodeOct {
  uint32_t nx, fx, ny, fy, nz, fz;
};

// OCT: every live ray of the packet has the same direction octant and pl6 holds the planes in
// {near x, far x, near y, far y, near z, far z} order (loaded through NodeOct offsets): the per-axis
// min/max pairs disappear. fma is monotone in the plane, so min(fma(lo), fma(hi)) IS the near
// plane's fma: the entry/exit distances, and so every decision and key, are bitwise those of the
// min/max form (dead rays, whatever their octant, still carry tbest = -inf and reject).
template <bool STATS, int R, bool OCT = false>
__device__ __forceinline__ uint32_t packet_slabs(const f4v (&pl6)[6], const PacketRay<R>& ry, float tmin,
                                                 const PacketLive<R>& pl, const HitRec* hit, uint32_t count,
                                                 uint64_t (&hm)[R][4], uint32_t (&vkey)[R][4], Counters& cnt) {
  const f4v a0 = pl6[0], a1 = pl6[1], a2 = pl6[2], a3 = pl6[3], a4 = pl6[4], a5 = pl6[5];
  const float lox[4] = {a0.x, a0.y, a0.z, a0.w}, hix[4] = {a1.x, a1.y, a1.z, a1.w};
  const float loy[4] = {a2.x, a2.y, a2.z, a2.w}, hiy[4] = {a3.x, a3.y, a3.z, a3.w};
  const float loz[4] = {a4.x, a4.y, a4.z, a4.w}, hiz[4] = {a5.x, a5.y, a5.z, a5.w};
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const V3 iv = ry.invd[r], no = ry.noinv[r];
    const float tbest = hit[r].t;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float tlx = __builtin_fmaf(lox[k], iv.x, no.x), thx = __builtin_fmaf(hix[k], iv.x, no.x);
      const float tly = __builtin_fmaf(loy[k], iv.y, no.y), thy = __builtin_fmaf(hiy[k], iv.y, no.y);
      const float tlz = __builtin_fmaf(loz[k], iv.z, no.z), thz = __builtin_fmaf(hiz[k], iv.z, no.z);
      float n, f;
      const float fzz = OCT ? thz : fmaxf(tlz, thz);
      float fz;
      // min with the loop-carried t: fminf would re-canonicalise t (a v_max t, t) at every node
      // visit; t is always a quiet value (arithmetic results and +-inf), so v_min gives its bits
      asm("v_min_f32 %0, %1, %2" : "=v"(fz) : "v"(fzz), "v"(tbest));
      if (OCT) {  // lo* hold the near planes, hi* the far planes
        n = fmaxf(fmaxf(tlx, tly), fmaxf(tlz, tmin));
        f = fminf(fminf(thx, thy), fz);
      } else {
        n = fmaxf(fmaxf(fminf(tlx, thx), fminf(tly, thy)), fmaxf(fminf(tlz, thz), tmin));
        f = fminf(fminf(fmaxf(tlx, thx), fmaxf(tly, thy)), fz);
      }
      const bool h = n <= f * 1.0000004f;  // only the lead's key is read
      hm[r][k] = wave_ballot(h);  // dead rays carry tbest = -inf: their h is false
      vkey[r][k] = __float_as_uint(h ? fabsf(n) : __builtin_inff());  // |n| folds into the select as a source modifier
    }
    if (STATS && ray_live(hit[r])) cnt.aabb += count;
  }
  uint64_t any[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    any[k] = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) any[k] |= hm[r][k];
  }
  return nonzero_mask4(any);
}

// TLAS node of the packet walk (children: TLAS nodes and instance leaves). The entered children go
// nearest first by the lead ray's entry distance (lowest slot on ties); the others are pushed in
// descending slot order, so the lowest slot pops next. Pushes that do not happen write the spare
// lane kPacketStack - 1; the bookkeeping is plain integer SALU work. Returns true with *next set,
// false when nothing is left to descend into.
template <bool ANY_HIT, bool STATS, int R>
__device__ __forceinline__ bool packet_tlas_node(const RT_CONST char* pool, int ref, const PacketRay<R>& ry,
                                                float tmin, PacketLive<R>& pl, const HitRec* hit, WaveStack& stk,
                                                int& sp, int cap, int& next, Counters& cnt) {
  const RT_CONST char* nb = pool + ((uint32_t)ref << 7);
  const i8v ch = *(const RT_CONST i8v*)(nb + 96);  // child[4], count, first_inner, inner_mask, pad
  const int cref[4] = {ch[0], ch[1], ch[2], ch[3]};
  if (STATS) ++cnt.nfetch;
  uint64_t hm[R][4];
  uint32_t vkey[R][4];
  const f4v planes[6] = {cld4(nb), cld4(nb + 16), cld4(nb + 32), cld4(nb + 48), cld4(nb + 64), cld4(nb + 80)};
  const uint32_t ent = packet_slabs<STATS, R>(planes, ry, tmin, pl, hit, (uint32_t)ch[4], hm, vkey, cnt);
  // pin the child-ref load before the early exit: issued with the plane loads, it shares their
  // scalar-cache round trip instead of starting a second one after the slab tests
  asm volatile("" ::"s"(ch[0]), "s"(ch[1]), "s"(ch[2]), "s"(ch[3]));
  if (ent == 0) return false;
  // nearest entered child by the lead ray's key, lowest slot on ties: per lane in VALU (keys
  // masked to the entered set), one readlane. Any-hit walks take the lowest entered slot.
  uint32_t ib;
  if (ANY_HIT || (ent & (ent - 1u)) == 0u) {  // no choice with one entered child
    ib = (uint32_t)__builtin_ctz(ent);
  } else {
    uint32_t idx = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      uint32_t kk[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) kk[k] = key_if_entered(vkey[r][k], ent, k);
      const uint32_t m = min(min(kk[0], kk[1]), min(kk[2], kk[3]));
      const uint32_t ir = kk[0] == m ? 0u : kk[1] == m ? 1u : kk[2] == m ? 2u : 3u;
      idx = (r == 0 || pl.lead_r == (uint32_t)r) ? ir : idx;
    }
    ib = (uint32_t)__builtin_amdgcn_readlane((int)idx, (int)pl.lead_l);
  }
  const i4v c4 = {ch[0], ch[1], ch[2], ch[3]};
  const int rb = c4[ib];
  // pushed set P (entered, not the nearest) as a 4-bit mask; descending slot order puts child k
  // at sp + popcount(P >> (k + 1)), so the four writes are independent of each other
  const uint32_t P = ent & ~(1u << ib);
  if (STATS && sp + __builtin_popcount(P) > cap)  // never: cap is the exact worst case
#pragma unroll
    for (int r = 0; r < R; ++r) cnt.overflow += ray_live(hit[r]) ? 1u : 0u;
  // a uniform branch per slot around its write (round 6: −1 … −3 % on every config against writing the slots not
  // pushed to the spare lane)
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if ((P >> k) & 1u) stk.put(sp + __builtin_popcount(P >> (k + 1)), cref[k]);
  sp = __builtin_amdgcn_readfirstlane(sp + __builtin_popcount(P));  // uniform by construction: an SGPR
  next = rb;
  return true;
}

#ifndef RT_HYBRID_T
#define RT_HYBRID_T 0  // packet BLAS nodes wanted by at most this many lanes go to per-lane walks (0: never)
#endif
#ifndef RT_HYBRID_ROOT
#define RT_HYBRID_ROOT 0  // 1: the hand-off is considered at a BLAS's root node only (one check per instance)
#endif
constexpr int kHybridLanes = RT_HYBRID_T > 0 ? RT_HYBRID_T : 1;  // LDS stack columns per wave
constexpr int kMaxPacketWaves = 2;                                // waves of a packet workgroup (packet_block)
#if RT_HYBRID_T
// the per-lane subtree stacks of a packet workgroup: one LDS array for every instantiation of the walk
// (a __shared__ inside the template would be allocated once per instantiation)
__shared__ int g_hyb[kMaxPacketWaves][kHybridStack * kHybridLanes];
#endif
#if RT_LDS_TOP
// RT_LDS_TOP experiment ("LDS node packets"): the first RT_LDS_TOP nodes (BFS order: the top levels)
// of the scene's largest BLAS, copied in by every packet workgroup at its start; the BLAS walk reads those nodes'
// planes from here (ds_read_b128, a broadcast of one address) instead of the scalar cache
__shared__ f4v g_top[RT_LDS_TOP * 8];
#endif

// Per-lane subtree walk inside the packet schedule (north star: wavefront ballot / prefix-sum ray
// compaction). A packet visits the union of its lanes' paths; when a BLAS node is wanted by few lanes
// (the ballot of lanes accepting any of its children), those lanes finish that node's subtree on their
// own: each lane takes a column of a small LDS stack by its prefix rank among them (mbcnt of the ballot:
// conflict-free, [entry][rank]), pushes its own accepted children nearest first and walks on with vector
// loads of the pool (the per-lane schedule's node visit: octant near / far rows, sort4, Moller-Trumbore).
// The wave then resumes the packet walk from its own stack. Results are the packet walk's: a lane visits
// every node and triangle of the subtree its own slab tests accept. tn: this lane's entry distances of the
// node's children (+inf: not accepted); refs: the node's child refs (pool node index, or ~triangle slot).
template <bool ANY_HIT, bool STATS>
__device__ __forceinline__ void lane_subtree(const RT_GLOBAL char* pn, const RT_GLOBAL char* pt, const int32_t* refs,
                                             const float* tn0, V3 ro, V3 rd, V3 rinvd, V3 rnoinv, float tmin,
                                             uint32_t cur, float face, HitRec& h, int* col, Counters& cnt) {
  float tn[4] = {tn0[0], tn0[1], tn0[2], tn0[3]};
  int32_t r[4] = {refs[0], refs[1], refs[2], refs[3]};
  sort4(tn, r);
  int sp = 0;
#pragma unroll
  for (int k = 3; k >= 1; --k)
    if (tn[k] != __builtin_inff()) col[(sp++) * kHybridLanes] = r[k];
  int ref = r[0];
  const Octant oct = octant(rinvd);
  while (true) {
    if (ref >= 0) {
      // slab tests axis by axis (two rows live at a time, not the node's 28 floats: the walk runs inside
      // the packet kernel's register budget). max / min are exact, so the regrouping gives
      // slab4_octant's entry / exit distances up to the sign of a zero, which no comparison sees.
      const uint32_t off = (uint32_t)ref << 7;
      f4v tn4, tf4;
      {
        const f4v a = ldf4(pn, off + oct.x), b = ldf4(pn, off + (oct.x ^ 16u));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          tn4[k] = __builtin_fmaf(a[k], rinvd.x, rnoinv.x);
          tf4[k] = __builtin_fmaf(b[k], rinvd.x, rnoinv.x);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      {
        const f4v a = ldf4(pn, off + oct.y), b = ldf4(pn, off + (oct.y ^ 16u));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          tn4[k] = fmaxf(tn4[k], __builtin_fmaf(a[k], rinvd.y, rnoinv.y));
          tf4[k] = fminf(tf4[k], __builtin_fmaf(b[k], rinvd.y, rnoinv.y));
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      const i4v ch = ldi4(pn, off + 96u);
      float t4[4];
      {
        const f4v a = ldf4(pn, off + oct.z), b = ldf4(pn, off + (oct.z ^ 16u));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float n = fmaxf(tn4[k], fmaxf(__builtin_fmaf(a[k], rinvd.z, rnoinv.z), tmin));
          const float f = fminf(tf4[k], fminf(__builtin_fmaf(b[k], rinvd.z, rnoinv.z), h.t));
          t4[k] = n <= f * 1.0000004f ? n : __builtin_inff();
        }
      }
      int32_t c[4] = {ch.x, ch.y, ch.z, ch.w};
      if (STATS) {
        ++cnt.lnfetch;
        cnt.aabb += (uint32_t)(c[0] != kEmptyChild) + (uint32_t)(c[1] != kEmptyChild) +
                    (uint32_t)(c[2] != kEmptyChild) + (uint32_t)(c[3] != kEmptyChild);
      }
      sort4(t4, c);
      if (t4[0] != __builtin_inff()) {
#pragma unroll
        for (int k = 3; k >= 1; --k)
          if (t4[k] != __builtin_inff()) col[(sp++) * kHybridLanes] = c[k];
        ref = c[0];
        continue;
      }
    } else {
      const uint32_t toff = (uint32_t)(~ref) * (uint32_t)sizeof(TriRec);
      const f4v a = ldf4(pt, toff), b = ldf4(pt, toff + 16u), c = ldf4(pt, toff + 32u);
      if (STATS) {
        ++cnt.tri;
        ++cnt.ltfetch;
      }
      float t, u, v;
      if (moller_trumbore(ro, rd, v3(a.x, a.y, a.z), v3(b.x, b.y, b.z), v3(c.x, c.y, c.z), face, t, u, v) &&
          t >= tmin) {
        const uint32_t prim = __float_as_uint(a.w);
        const bool better = ANY_HIT ? (t <= h.t)
                                    : (t < h.t || (t == h.t && (cur < h.inst || (cur == h.inst && prim < h.prim))));
        if (better) {
          h.t = ANY_HIT ? -__builtin_inff() : t;  // an any-hit ray leaves with t = -inf, as in the packet
          h.u = u;
          h.v = v;
          h.inst = cur;
          h.prim = prim;
          if (ANY_HIT) return;
        }
      }
    }
    if (sp == 0) return;
    ref = col[(--sp) * kHybridLanes];
  }
}

// BLAS walk of the packet (instance cur, object rays ry) on the stack above `base`; returns false
// when an any-hit packet has no live ray left. One loop iteration per node, straight-line uniform
// control flow (no status codes between a node function and the loop). At a node: entered
// triangle children are tested right here, in slot order; of the entered internal children the
// nearest (the lead ray's entry distance, lowest slot on ties; chosen per lane in VALU, one
// readlane; any-hit walks take the lowest entered slot) is descended into, and the rest become ONE
// stack entry (first_inner << 8 | inner_mask << 4 | pending slots) that pops its slots lowest
// first — exactly the order in which per-child pushes in descending slot order would pop them, so
// the walk (and every counter) is that of the per-child stack with a fraction of the scalar
// bookkeeping. BLAS nodes hold their internal children in the lowest slots, so the internal child in
// slot k is first_inner + k.
template <bool ANY_HIT, bool STATS, int R, bool OCT>
__device__ __forceinline__ bool packet_blas_walk(const RT_CONST char* pool, const RT_CONST TriRec* tpool, int bref,
                                                 const PacketRay<R>& ry, float tmin, uint32_t cur, float face,
                                                 PacketLive<R>& pl, HitRec* hit, WaveStack& stk, int& sp, int cap,
                                                 const NodeOct& oc, int hybrid, int lds_root, int lds_n,
                                                 Counters& cnt) {
  (void)lds_root;
  (void)lds_n;
  const int base = sp;
#if RT_HYBRID_T
  // the same pools for per-lane (vector) loads in lane_subtree
  const RT_GLOBAL char* gpool = (const RT_GLOBAL char*)pool;
  const RT_GLOBAL char* gtpool = (const RT_GLOBAL char*)tpool;
#else
  (void)hybrid;
#endif
  while (true) {
    const RT_CONST char* nb = pool + ((uint32_t)bref << 7);
    const i8v ch = *(const RT_CONST i8v*)(nb + 96);  // child[4], count, first_inner, inner_mask, entry_base
    if (STATS) ++cnt.nfetch;
    uint64_t hm[R][4];
    uint32_t vkey[R][4];
    f4v planes[6];
    uint32_t ent;
#if RT_LDS_TOP
    const uint32_t rel = (uint32_t)(bref - lds_root);
    if (rel < (uint32_t)lds_n) {
      // rows at the octant offsets (or in order), from LDS into VGPRs; a separate slab call so the scalar path's
      // SGPR planes are not merged into VGPRs
      const char* sn = (const char*)g_top + (rel << 7);
      f4v lp[6];
      if (OCT) {
        lp[0] = *(const f4v*)(sn + oc.nx);
        lp[1] = *(const f4v*)(sn + oc.fx);
        lp[2] = *(const f4v*)(sn + oc.ny);
        lp[3] = *(const f4v*)(sn + oc.fy);
        lp[4] = *(const f4v*)(sn + oc.nz);
        lp[5] = *(const f4v*)(sn + oc.fz);
      } else {
#pragma unroll
        for (int q = 0; q < 6; ++q) lp[q] = *(const f4v*)(sn + 16 * q);
      }
      ent = packet_slabs<STATS, R, OCT>(lp, ry, tmin, pl, hit, (uint32_t)ch[4], hm, vkey, cnt);
    } else
#endif
    {
    if (OCT) {
      // one 32-bit offset per row: the scalar load takes it as its SGPR offset (no 64-bit adds)
      const uint32_t noff = (uint32_t)bref << 7;
      // each row at the pool base + its octant offset (SGPR soffset) + the node offset as the
      // instruction's... the node offset goes into the base once (two SALU); six s_load_dwordx4 with
      // the row offsets as soffset (the compiler would add 64-bit addresses per row itself)
      const RT_CONST char* nbo = pool + noff;
      asm volatile(
          "s_load_dwordx4 %0, %6, %7\n\t"
          "s_load_dwordx4 %1, %6, %8\n\t"
          "s_load_dwordx4 %2, %6, %9\n\t"
          "s_load_dwordx4 %3, %6, %10\n\t"
          "s_load_dwordx4 %4, %6, %11\n\t"
          "s_load_dwordx4 %5, %6, %12\n\t"
          "s_waitcnt lgkmcnt(0)"
          : "=&s"(planes[0]), "=&s"(planes[1]), "=&s"(planes[2]), "=&s"(planes[3]), "=&s"(planes[4]),
            "=&s"(planes[5])
          : "s"(nbo), "s"(oc.nx), "s"(oc.fx), "s"(oc.ny), "s"(oc.fy), "s"(oc.nz), "s"(oc.fz)
          : "memory");
    } else {
#pragma unroll
      for (int q = 0; q < 6; ++q) planes[q] = cld4(nb + 16 * q);
    }
    ent = packet_slabs<STATS, R, OCT>(planes, ry, tmin, pl, hit, (uint32_t)ch[4], hm, vkey, cnt);
    }
    asm volatile("" ::"s"(ch[0]), "s"(ch[1]), "s"(ch[2]), "s"(ch[3]), "s"(ch[5]), "s"(ch[6]), "s"(ch[7]));
#if RT_HYBRID_T
    // few lanes want this node: they walk its subtree on their own (lane_subtree), then the packet pops
    if (R == 1 && hybrid && (ent & (uint32_t)ch[6]) != 0u && (!RT_HYBRID_ROOT || sp == base)) {
      const uint64_t act = (hm[0][0] | hm[0][1]) | (hm[0][2] | hm[0][3]);
      if (__builtin_popcountll(act) <= RT_HYBRID_T) {
        const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
        const uint32_t rank =
            __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
        if ((act >> (threadIdx.x & 63u)) & 1ull) {
          const float tn[4] = {__uint_as_float(vkey[0][0]), __uint_as_float(vkey[0][1]), __uint_as_float(vkey[0][2]),
                               __uint_as_float(vkey[0][3])};
          const int32_t refs[4] = {ch[0], ch[1], ch[2], ch[3]};
          lane_subtree<ANY_HIT, STATS>(gpool, gtpool, refs, tn, ry.o[0], ry.d[0], ry.invd[0], ry.noinv[0], tmin, cur,
                                       face, hit[0], &g_hyb[w][rank], cnt);
        }
        if (ANY_HIT && !pl.update(hit)) return false;
        if (sp == base) return true;
        bref = pop_entry(stk.v, sp);
        continue;
      }
    }
#endif
    const uint32_t imask = (uint32_t)ch[6];
    uint32_t tl = ent & ~imask;
    ent &= imask;
    if (tl) {
      // one test per slot with the slot's ref in a fixed SGPR (no ref-select chain, no loop)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (tl & (1u << k)) {
          uint64_t own[R];
#pragma unroll
          for (int r = 0; r < R; ++r) own[r] = hm[r][k];
          packet_tri<ANY_HIT, STATS, R>(tpool, ch[k], ry, tmin, cur, face, pl, hit, own, cnt);
        }
      if (ANY_HIT) {  // rays can only have left the packet in a triangle test
        if (!pl.update(hit)) return false;
        // children only finished rays wanted are dropped
        uint64_t any[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          any[k] = 0;
#pragma unroll
          for (int r = 0; r < R; ++r) any[k] |= hm[r][k] & pl.mask[r];
        }
        ent &= nonzero_mask4(any);
      }
    }
    if (ent) {
      uint32_t ib, nref;
      if (ANY_HIT || (ent & (ent - 1u)) == 0u) {
        // occlusion rays skip the nearest-first choice (no keys, no readlane): for an occlusion ray
        // the order only decides how soon it stops; a closest-hit node with ONE entered internal
        // child has no choice to make
        ib = (uint32_t)__builtin_ctz(ent);
        nref = (uint32_t)ch[5] + ib;  // internal children in the lowest slots
      } else {
        // per lane: the slot of its smallest key over the entered internal children (all-ones
        // keys elsewhere), lowest slot on ties, and that child's ref (first_inner + slot: internal
        // children sit in the lowest slots), packed as ref << 2 | slot; the lead lane's answer, one
        // readlane, is the packet's
        uint32_t idx = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          uint32_t kk[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) kk[k] = key_if_entered(vkey[r][k], ent, k);
          const uint32_t m = min(min(kk[0], kk[1]), min(kk[2], kk[3]));
          const uint32_t ir = kk[0] == m ? 0u : kk[1] == m ? 1u : kk[2] == m ? 2u : 3u;
          const uint32_t pr = (((uint32_t)ch[5] + ir) << 2) | ir;
          idx = (r == 0 || pl.lead_r == (uint32_t)r) ? pr : idx;
        }
        const uint32_t pk = (uint32_t)__builtin_amdgcn_readlane((int)idx, (int)pl.lead_l);
        ib = pk & 3u;
        nref = pk >> 2;
      }
      if (STATS && (ent & ~(1u << ib)) && sp + 1 > cap)  // never: cap bounds the entries (one per level)
#pragma unroll
        for (int r = 0; r < R; ++r) cnt.overflow += ray_live(hit[r]) ? 1u : 0u;
      stk.v = push_entry(stk.v, sp, (uint32_t)ch[7], ent, 1u << ib);
      bref = (int)nref;
    } else {
      if (sp == base) return true;
      // top entry: its lowest pending slot is next; the entry stays while slots remain
      bref = pop_entry(stk.v, sp);
    }
  }
}

// The walk of trace_packet. Rays that are not alive start with t = -inf, so every slab test
// rejects them and the ballots need no live mask.
template <bool ANY_HIT, bool STATS, int R, bool CULL>
__device__ __forceinline__ void packet_walk(const SceneView& sc, const V3* o, const V3* d, float tmin, float tmax,
                                            const bool* alive, HitRec* hit, Counters& cnt) {
  const RT_CONST char* pool = (const RT_CONST char*)sc.pool_nodes;
  const RT_CONST TriRec* tpool = (const RT_CONST TriRec*)sc.pool_tris;
  const RT_CONST InstanceRec* ipool = (const RT_CONST InstanceRec*)sc.inst;
  PacketLive<R> pl;
  PacketRay<R> w;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    hit[r].t = alive[r] ? tmax : -__builtin_inff();
    hit[r].inst = 0xffffffffu;
    hit[r].prim = 0xffffffffu;
    hit[r].u = hit[r].v = 0.0f;
    w.o[r] = o[r];
    w.d[r] = d[r];
    w.invd[r] = v3(safe_inv(d[r].x), safe_inv(d[r].y), safe_inv(d[r].z));
    w.noinv[r] = neg(mul(o[r], w.invd[r]));
  }
  if (!pl.update(hit)) return;
  WaveStack stk;
  const int cap = sc.packet_cap;  // < kPacketStack (checked at launch): lane 63 stays spare
  int sp = 0;
  int ref = sc.tlas_root;
  // TLAS walk; each instance leaf runs a nested BLAS walk on the stack above the TLAS entries
  // (the world rays are invariant here, the object rays inside: no ray state moves around).
  while (true) {
    bool descend = false;
    if (ref >= 0) {
      int next;
      descend = packet_tlas_node<ANY_HIT, STATS, R>(pool, ref, w, tmin, pl, hit, stk, sp, cap, next, cnt);
      ref = descend ? next : ref;
    } else {
      const uint32_t cur = (uint32_t)(~ref);
      const RT_CONST InstanceRec& ir = ipool[cur];
      const RT_CONST f4v* mq = (const RT_CONST f4v*)ir.w2o;
      const f4v m0 = mq[0], m1 = mq[1], m2 = mq[2];
      const float m[12] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w, m2.x, m2.y, m2.z, m2.w};
      if (STATS) ++cnt.ifetch;
      PacketRay<R> b;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (STATS && ray_live(hit[r])) ++cnt.inst;
        if (ir.translate) {  // uniform: origin moved, direction and its inverse are the world ray's
          b.o[r] = inst_point(m, 1u, o[r]);
          b.d[r] = d[r];
          b.invd[r] = w.invd[r];
        } else {
          b.o[r] = xform_point(m, o[r]);
          b.d[r] = xform_dir(m, d[r]);
          b.invd[r] = v3(safe_inv(b.d[r].x), safe_inv(b.d[r].y), safe_inv(b.d[r].z));
        }
        b.noinv[r] = neg(mul(b.o[r], b.invd[r]));
      }
      const float face = CULL ? (ir.flip ? -1.0f : 1.0f) * sc.cull_sense : 0.0f;
      // one direction octant for every live object ray: near/far planes picked by load offsets
      bool uni = false;
      NodeOct oc{0u, 16u, 32u, 48u, 64u, 80u};
#if RT_PACKET_OCT
      if (R == 1) {
        const uint64_t live = pl.mask[0];
        const uint64_t sx = wave_ballot((int)__float_as_uint(b.invd[0].x) < 0) & live;
        const uint64_t sy = wave_ballot((int)__float_as_uint(b.invd[0].y) < 0) & live;
        const uint64_t sz = wave_ballot((int)__float_as_uint(b.invd[0].z) < 0) & live;
        uni = (sx == 0 || sx == live) && (sy == 0 || sy == live) && (sz == 0 || sz == live);
        const uint32_t ox = sx ? 16u : 0u, oy = sy ? 16u : 0u, oz = sz ? 16u : 0u;
        oc = NodeOct{ox, 16u - ox, 32u + oy, 48u - oy, 64u + oz, 80u - oz};
      }
#endif
#if RT_LDS_TOP
      const int lroot = sc.lds_root, ln = sc.lds_n;
#else
      const int lroot = 0, ln = 0;
#endif
      const bool more = uni ? packet_blas_walk<ANY_HIT, STATS, R, true>(pool, tpool, (int)ir.pool_root, b, tmin, cur,
                                                                          face, pl, hit, stk, sp, cap, oc, sc.hybrid,
                                                                          lroot, ln, cnt)
                            : packet_blas_walk<ANY_HIT, STATS, R, false>(pool, tpool, (int)ir.pool_root, b, tmin,
                                                                           cur, face, pl, hit, stk, sp, cap, oc, sc.hybrid,
                                                                           lroot, ln, cnt);
      if (ANY_HIT && !more) return;
    }
    if (!descend) {
      if (sp == 0) return;
      ref = stk.get(--sp);
    }
  }
}

// Traces the R rays of every lane (o, d, alive per slot) as one packet; found[r] / hit[r] per ray
// (a ray found a hit iff one was accepted: inst is set on acceptance only). Any-hit rays report
// acceptance only (t is -inf once accepted).
template <bool ANY_HIT, bool STATS, int R, bool CULL = false>
__device__ void trace_packet(const SceneView& sc, const V3* o, const V3* d, float tmin, float tmax,
                             const bool* alive, bool* found, HitRec* hit, Counters& cnt) {
  packet_walk<ANY_HIT, STATS, R, CULL>(sc, o, d, tmin, tmax, alive, hit, cnt);
#pragma unroll
  for (int r = 0; r < R; ++r) found[r] = hit[r].inst != 0xffffffffu;
}

// Hit-instance data the shaders read (the reference binds it per hit group through the SBT).
struct HitInstance {
  const RT_GLOBAL float* vtx;
  const RT_GLOBAL uint32_t* idx;
  float nrm[9];
  uint32_t hit_group;
  uint32_t instance_id;  // InstanceID(): reflective when 0 or 1 (Hit.hlsl:196)
};

__device__ __forceinline__ HitInstance load_hit_instance(const SceneView& sc, uint32_t inst) {
  const RT_GLOBAL InstanceRec* ir = gp(sc.inst) + inst;
  HitInstance h;
  h.vtx = gp(ir->vtx);
  h.idx = gp(ir->idx);
  for (int k = 0; k < 9; ++k) h.nrm[k] = ir->nrm[k];
  h.hit_group = ir->hit_group;
  h.instance_id = ir->instance_id;
  return h;
}

__device__ __forceinline__ V3 ldg3(const RT_GLOBAL float* p) { return v3(p[0], p[1], p[2]); }

__device__ __forceinline__ void tri_vertex_ids(const HitInstance& hi, uint32_t prim, uint32_t& i0, uint32_t& i1,
                                               uint32_t& i2) {
  if (hi.idx) {
    i0 = hi.idx[3 * prim];
    i1 = hi.idx[3 * prim + 1];
    i2 = hi.idx[3 * prim + 2];
  } else {
    i0 = 3 * prim;
    i1 = 3 * prim + 1;
    i2 = 3 * prim + 2;
  }
}

// normalize with its 1 / sqrt by rcp_exact when EX (the IEEE 1.0f / x, bit for bit: the same vector). Used on the REF
// shading's paths only: in the Lambert kernels the extra uniform branch of rcp_exact's slow path costs more than the
// division it replaces (RT_RCP_EXACT), in the REF kernels it pays.
template <bool EX>
__device__ __forceinline__ V3 normalize_x(V3 a) {
  if (EX) return muls(a, rcp_exact(sqrtf(dot(a, a))));
  return normalize(a);
}

// CalculateInterpolatedWorldNormal (Hit.hlsl:67-81): vertex order 1,2,0 against (u, v, 1-u-v).
template <bool EX = false>
__device__ V3 interpolated_world_normal(const HitInstance& hi, uint32_t prim, float u, float v) {
  uint32_t i0, i1, i2;
  tri_vertex_ids(hi, prim, i0, i1, i2);
  const V3 n0 = ldg3(hi.vtx + (size_t)i1 * 6 + 3);
  const V3 n1 = ldg3(hi.vtx + (size_t)i2 * 6 + 3);
  const V3 n2 = ldg3(hi.vtx + (size_t)i0 * 6 + 3);
  const float bz = (1.0f - u) - v;
  V3 n = normalize_x<EX>(add(add(muls(n0, u), muls(n1, v)), muls(n2, bz)));
  n = mat3_mul(hi.nrm, n);
  return normalize_x<EX>(n);
}

// PlaneClosestHit face normal (Hit.hlsl:218-222): normalize(cross(e1, e2)), then the instance
// normal matrix without renormalisation.
template <bool EX = false>
__device__ V3 face_world_normal(const HitInstance& hi, uint32_t prim) {
  uint32_t i0, i1, i2;
  tri_vertex_ids(hi, prim, i0, i1, i2);
  const V3 p0 = ldg3(hi.vtx + (size_t)i0 * 6);
  const V3 p1 = ldg3(hi.vtx + (size_t)i1 * 6);
  const V3 p2 = ldg3(hi.vtx + (size_t)i2 * 6);
  V3 n = normalize_x<EX>(cross(sub(p1, p0), sub(p2, p0)));
  return mat3_mul(hi.nrm, n);
}


// ClosestHit's finalSurfaceColor = CalculateDirectLighting (Hit.hlsl:83-95) + CalculatePBRShading
// (:97-174), pinned for float32 and mirrored bit for bit by oracle/rt_oracle.c osurface (round 6):
//  * ONE loop over the lights: the direct term's -normalize(lp - P) and the PBR term's L and distance
//    share one sqrt and one reciprocal (normalize is v * (1 / sqrt(dot v v)), length that same sqrt);
//    the two sums keep their own accumulators and light order, and are added at the end as before;
//  * the pixel's invariants (N, V, N.V, Smith's view term) out of the loop, the material's (a^2, k,
//    F0, (1 - metallic) albedo / PI) evaluated once per rt_set_shading on the host (FrameParams::surf);
//  * every quotient as a product with a reciprocal (rcp_exact: the IEEE 1.0f / x, bits and all):
//    NDF = a2 * (1 / denom), Smith's light term NdotL * (1 / (NdotL (1 - k) + k)), the specular
//    term F * ((NDF G) * (1 / (4 N.V N.L + 1e-4))), the tone map c * (1 / (c + 1)); the diffuse
//    term (1 - F) * ((1 - metallic) albedo / PI).
// Against the float64 restatement (oracle/np_reference.py) this changes nothing measurable (the
// goldens' L-inf stays <= 1e-4); against the HLSL it is as faithful as the IEEE quotients were,
// since DXC compiles HLSL divisions to reciprocal products itself.
__device__ __forceinline__ float srcp(float x) { return rcp_exact(x); }

__device__ V3 surface_ref(const FrameParams& fp, V3 P, V3 n, V3 cam) {
  const MaterialRec& m = fp.material;
  const V3 albedo = v3(m.albedo[0], m.albedo[1], m.albedo[2]);
  // the material's constants, from rt_set_shading (surface_consts: the same IEEE operations on the host, the same
  // bits; per pixel they were three divisions and a dozen products: REF -1.5 %, REFL -6 %, frames bit-equal)
  const float a2 = fp.surf.a2, k = fp.surf.k, omk = fp.surf.omk;
  const V3 F0 = v3(fp.surf.F0[0], fp.surf.F0[1], fp.surf.F0[2]);
  const V3 kdA = v3(fp.surf.kdA[0], fp.surf.kdA[1], fp.surf.kdA[2]);
  const V3 N = neg(muls(n, srcp(sqrtf(dot(n, n)))));
  const V3 Vd = sub(cam, P);
  const V3 V = muls(Vd, srcp(sqrtf(dot(Vd, Vd))));
  const float NdotV = maxf(dot(N, V), 0.0f);
  const float ggx2 = NdotV * srcp(NdotV * omk + k);
  const float v4 = 4.0f * NdotV;
  V3 cd = v3(0.0f, 0.0f, 0.0f), L0 = v3(0.0f, 0.0f, 0.0f);
  for (uint32_t l = 0; l < fp.nlights; ++l) {
    const LightRec& Lr = fp.lights[l];
    const V3 lp = v3(Lr.position[0], Lr.position[1], Lr.position[2]);
    const V3 lc = v3(Lr.color[0], Lr.color[1], Lr.color[2]);
    const V3 dv = sub(lp, P);
    const float dist = sqrtf(dot(dv, dv));
    const V3 L = muls(dv, srcp(dist));
    // CalculateDirectLighting
    const float ti = maxf(0.0f, dot(n, neg(L)) * Lr.intensity);
    cd = add(cd, muls(mul(albedo, lc), ti));
    // CalculatePBRShading
    const V3 Hd = add(V, L);
    const V3 H = muls(Hd, srcp(sqrtf(dot(Hd, Hd))));
    const float att = srcp(maxf(dist * dist, 1.0f));
    const V3 radiance = muls(lc, att);
    const float x = clamp01(1.0f - maxf(dot(H, V), 0.0f));
    const float x2 = x * x;
    const float x5 = (x2 * x2) * x;
    const V3 F = v3(F0.x + (1.0f - F0.x) * x5, F0.y + (1.0f - F0.y) * x5, F0.z + (1.0f - F0.z) * x5);
    const float NdotH = maxf(dot(N, H), 0.0f);
    const float NdotH2 = NdotH * NdotH;
    float denom = NdotH2 * (a2 - 1.0f) + 1.0f;
    denom = (kPi * denom) * denom;
    const float NDF = a2 * srcp(denom);
    const float NdotL = maxf(dot(N, L), 0.0f);
    const float ggx1 = NdotL * srcp(NdotL * omk + k);
    const float G = ggx1 * ggx2;
    const float sp = (NDF * G) * srcp(v4 * NdotL + 0.0001f);
    const V3 spec = muls(F, sp);
    const V3 diff = v3((1.0f - F.x) * kdA.x, (1.0f - F.y) * kdA.y, (1.0f - F.z) * kdA.z);
    L0 = add(L0, muls(mul(add(diff, spec), radiance), NdotL));
  }
  V3 c = muls(L0, 0.2f);
  c = v3(c.x * srcp(c.x + 1.0f), c.y * srcp(c.y + 1.0f), c.z * srcp(c.z + 1.0f));
  const float g = 1.0f / 2.2f;
  return add(cd, v3(det_pow(c.x, g), det_pow(c.y, g), det_pow(c.z, g)));
}

template <bool STATS>
__device__ bool shadow_ray(const SceneView& sc, V3 P, V3 dir, const LaneStack& stk, Counters& cnt) {
  HitRec h;
  if (STATS) ++cnt.shadow;
  return trace<true, STATS>(sc, P, normalize(dir), 0.01f, 100000.0f, h, stk, cnt);
}

__device__ __forceinline__ V3 miss_color(const FrameParams& fp, uint32_t py) {
  const float ramp = (float)py / fp.fheight;  // Miss.hlsl:8 (DispatchRaysIndex: the pixel row at every depth)
  return v3(0.0f, 0.2f, 0.7f - 0.3f * ramp);
}

// ReflectRay + CastReflectionRay (Hit.hlsl:176-181, Common.hlsl:58-69): the reflected direction
// (normalised three times, as the HLSL does) and the offset origin.
__device__ __forceinline__ void reflection_ray(V3 P, V3 n, V3 rd, V3& ro_next, V3& rd_next) {
  const V3 dir = normalize_x<true>(normalize_x<true>(reflect_dir(normalize_x<true>(rd), n)));
  ro_next = add(P, muls(dir, 0.001f));
  rd_next = dir;
}

__device__ __forceinline__ bool reflective(const FrameParams& fp, const HitInstance& ir, int depth) {
  return fp.material.reflectivity != 0.0f && (ir.instance_id == 0u || ir.instance_id == 1u) &&
         depth < kMaxReflectDepth;
}

// HLSL lerp(x, y, s) = x + s * (y - x).
__device__ __forceinline__ V3 lerp3(V3 x, V3 y, float s) {
  return v3(x.x + s * (y.x - x.x), x.y + s * (y.y - x.y), x.z + s * (y.z - x.z));
}

// The payload colour of a reflection chain as the HLSL recursion returns it: each ClosestHit
// level k sets lerp(s_k, <colour of level k + 1>, r) after its nested TraceRay returned
// (Hit.hlsl:194-203), so the innermost lerp is evaluated first. sk[0..n) holds the levels'
// own surface colours (finalSurfaceColor), c the colour the innermost ray came back with.
__device__ __forceinline__ V3 unwind_chain(const V3* sk, int n, V3 c, float r) {
  for (int k = n - 1; k >= 0; --k) c = lerp3(sk[k], c, r);
  return c;
}

// RT_SHADE_REF for one camera ray, one lane: ClosestHit (Hit.hlsl:183-204) / PlaneClosestHit
// (:207-241) / Miss, with the reflection rays of InstanceID 0 and 1 when the material's
// reflectivity r != 0 (back faces culled). Each level's surface colour is kept (per-lane
// scratch, touched only by reflective hits) and the nested lerps are unwound innermost first,
// as the recursion evaluates them (oracle/rt_oracle.c oshade_ref mirrors it). r == 0 traces no
// reflection.
template <bool STATS>
__device__ V3 shade_ref(const SceneView& sc, const FrameParams& fp, uint32_t py, V3 O, V3 D, bool f, HitRec hit,
                        const LaneStack& stk, Counters& cnt) {
  const float refl = fp.material.reflectivity;
  V3 sk[kMaxReflectDepth];
  V3 ro = O, rd = D;
  for (int depth = 0;; ++depth) {
    V3 term;
    if (!f) {
      term = miss_color(fp, py);
    } else {
      const HitInstance ir = load_hit_instance(sc, hit.inst);
      const V3 P = add(ro, muls(rd, hit.t));  // GetWorldHitPoint, Common.hlsl:24-27
      if (ir.hit_group == 2u) {
        const LightRec& L0 = fp.lights[0];
        const V3 ldir = normalize(sub(v3(L0.position[0], L0.position[1], L0.position[2]), P));
        const V3 n = face_world_normal(ir, hit.prim);
        bool shadowed = dot(n, ldir) < 0.0f;
        const bool occl = shadow_ray<STATS>(sc, P, ldir, stk, cnt);
        if (!shadowed) shadowed = occl;
        const float factor = shadowed ? 0.3f : 1.0f;
        const float li = maxf(0.0f, dot(n, ldir));
        const float c = (1.0f * li) * factor;
        term = v3(c, c, c);
      } else {
        const V3 n = interpolated_world_normal(ir, hit.prim, hit.u, hit.v);
        const V3 s = surface_ref(fp, P, n, ro);
        if (reflective(fp, ir, depth)) {
          sk[depth] = s;
          reflection_ray(P, n, rd, ro, rd);
          if (STATS) ++cnt.refl;
          f = trace<false, STATS, true>(sc, ro, rd, 0.001f, 1000.0f, hit, stk, cnt);
          continue;
        }
        term = s;
      }
    }
    return unwind_chain(sk, depth, term, refl);
  }
}

// One camera sample -> color (RayGen.hlsl:28-43 and the hit/miss programs).
template <int MODE, bool STATS>
__device__ V3 shade_sample(const SceneView& sc, const FrameParams& fp, const FrameCam& cam, uint32_t px, uint32_t py,
                           float ox, float oy, const LaneStack& stk, Counters& cnt) {
  const float dx = (((float)px + ox) / fp.fwidth) * 2.0f - 1.0f;
  const float dy = (((float)py + oy) / fp.fheight) * 2.0f - 1.0f;
  float dc[4], dw[4];
  const float ndc[4] = {dx, -dy, 1.0f, 1.0f};
  hlsl_mul4(cam.proj_inv, ndc, dc);
  const float dcam[4] = {dc[0], dc[1], dc[2], 0.0f};
  hlsl_mul4(cam.view_inv, dcam, dw);
  const V3 O = v3(cam.origin[0], cam.origin[1], cam.origin[2]);  // mul(viewInverse, (0,0,0,1))
  const V3 D = normalize(v3(dw[0], dw[1], dw[2]));  // CastDefaultRay
  HitRec hit;
  if (STATS) ++cnt.primary;
  const bool f = trace<false, STATS>(sc, O, D, 0.0f, 100000.0f, hit, stk, cnt);
  if (MODE == 0 || MODE == 3) return shade_ref<STATS>(sc, fp, py, O, D, f, hit, stk, cnt);
  if (!f) return miss_color(fp, py);
  const HitInstance ir = load_hit_instance(sc, hit.inst);
  const V3 P = add(O, muls(D, hit.t));  // GetWorldHitPoint, Common.hlsl:24-27
  const bool plane = ir.hit_group == 2u;
  // RT_SHADE_LAMBERT_SHADOW (MODE 1) and RT_SHADE_PRIMARY (MODE 2)
  const V3 n = plane ? face_world_normal(ir, hit.prim) : neg(interpolated_world_normal(ir, hit.prim, hit.u, hit.v));
  float c = 0.0f;
  for (uint32_t l = 0; l < fp.nlights; ++l) {
    const LightRec& Lr = fp.lights[l];
    const V3 L = normalize(sub(v3(Lr.position[0], Lr.position[1], Lr.position[2]), P));
    const float nl = dot(n, L);
    if (nl > 0.0f) {
      float factor = 1.0f;
      if (MODE == 1 && shadow_ray<STATS>(sc, P, L, stk, cnt)) factor = 0.3f;
      c = c + nl * factor;
    }
  }
  c = c / (float)fp.nlights;
  return v3(c, c, c);
}

#ifndef RT_SHADOW_COMPACT
#define RT_SHADOW_COMPACT 0  // workgroup shadow-ray compaction (measured: not a win)
#endif

// Workgroup ray compaction of one light's shadow rays (north star: "wavefront ballot/prefix-sum for
// ray compaction"): each wave ballots its lanes that need the ray, the waves' counts go through
// LDS, and when all of them fit one 64-ray packet (and more than one wave has some) the rays are
// compacted — slot = the wave's prefix + mbcnt of the ballot — and wave 0 traces them as ONE packet,
// the occlusion bits coming back through LDS; otherwise every wave traces its own packet. The
// whole workgroup must call it (uniform per light: two barriers). Same results as the per-wave
// packets (a ray's occlusion does not depend on its packet). Kept as RT_SHADOW_COMPACT: with the
// screen-tile waves the shadow packets are already ~94-99 % full (C2-C4), so it rarely fires.
template <bool STATS>
__device__ bool shadow_compact(const SceneView& sc, V3 P, V3 d, bool need, uint32_t parity, Counters& cnt) {
  __shared__ float s_ray[6][64];
  __shared__ uint32_t s_cnt[2][4];
  __shared__ uint32_t s_occ[2];
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint64_t m = wave_ballot(need);
  if (lane == 0) s_cnt[parity][w] = (uint32_t)__builtin_popcountll(m);
  __syncthreads();
  uint32_t total = 0, base = 0, busy = 0;
  for (uint32_t k = 0; k < nw; ++k) {
    const uint32_t c = s_cnt[parity][k];
    base += k < w ? c : 0u;
    total += c;
    busy += c ? 1u : 0u;
  }
  const bool merge = total <= 64u && busy >= 2u;  // uniform over the workgroup
  const uint32_t slot = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  V3 q = P, e = d;
  bool alive = need;
  if (merge) {
    if (need) {
      s_ray[0][slot] = P.x;
      s_ray[1][slot] = P.y;
      s_ray[2][slot] = P.z;
      s_ray[3][slot] = d.x;
      s_ray[4][slot] = d.y;
      s_ray[5][slot] = d.z;
    }
    __syncthreads();
    alive = w == 0 && lane < total;
    if (alive) {
      q = v3(s_ray[0][lane], s_ray[1][lane], s_ray[2][lane]);
      e = v3(s_ray[3][lane], s_ray[4][lane], s_ray[5][lane]);
    }
  }
  // one packet per wave, or the merged packet in wave 0 (the other waves' packets are all dead and
  // return at once); a single inlined walk keeps the kernel's registers
  HitRec h;
  bool f;
  trace_packet<true, STATS, 1>(sc, &q, &e, 0.01f, 100000.0f, &alive, &f, &h, cnt);
  if (!merge) return f;
  const uint64_t om = wave_ballot(f);
  if (w == 0 && lane == 0) {
    s_occ[0] = (uint32_t)om;
    s_occ[1] = (uint32_t)(om >> 32);
  }
  __syncthreads();
  return need && ((s_occ[slot >> 5] >> (slot & 31u)) & 1u) != 0u;
}

// shade_sample for the wave-packet traversal: identical arithmetic per ray, with every trace
// hoisted to wave-uniform control flow (rays without a trace of that kind join the packet dead).
// Each lane shades R camera samples (R pixels) at once.
#ifndef RT_WAVE_TIMES
#define RT_WAVE_TIMES 0  // 1: every wave stores its start / end clock (diagnostics; tools/wave_times.py)
#endif
template <int MODE, bool STATS, int R>
__device__ void shade_sample_packet(const SceneView& sc, const FrameParams& fp, const FrameCam& cam, const uint32_t* px,
                                    const uint32_t* py, float ox, float oy, const bool* inimg, V3* color,
                                    Counters& cnt) {
  V3 O[R], D[R], P[R], sd[R];
  HitRec hit[R], sh[R];
  bool found[R], occl[R], need[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const float dx = (((float)px[r] + ox) / fp.fwidth) * 2.0f - 1.0f;
    const float dy = (((float)py[r] + oy) / fp.fheight) * 2.0f - 1.0f;
    float dc[4], dw[4];
    const float ndc[4] = {dx, -dy, 1.0f, 1.0f};
    hlsl_mul4(cam.proj_inv, ndc, dc);
    const float dcam[4] = {dc[0], dc[1], dc[2], 0.0f};
    hlsl_mul4(cam.view_inv, dcam, dw);
    O[r] = v3(cam.origin[0], cam.origin[1], cam.origin[2]);  // mul(viewInverse, (0,0,0,1))
    D[r] = normalize(v3(dw[0], dw[1], dw[2]));  // CastDefaultRay
    if (STATS && inimg[r]) ++cnt.primary;
  }
  trace_packet<false, STATS, R>(sc, O, D, 0.0f, 100000.0f, inimg, found, hit, cnt);
#pragma unroll
  for (int r = 0; r < R; ++r) P[r] = add(O[r], muls(D[r], hit[r].t));  // GetWorldHitPoint, Common.hlsl:24-27
  if (MODE == 0 || MODE == 3) {  // MODE 3: RT_SHADE_REF with reflectivity 0 (no reflection rays)
#pragma unroll
    for (int r = 0; r < R; ++r) color[r] = miss_color(fp, py[r]);
    // shade_ref level by level for the whole packet: each level's shadow rays and next
    // reflection rays are one packet each (mirrored by oracle osample_packet)
    const float refl = fp.material.reflectivity;
    V3 ro[R], rd[R], ldir[R], nf[R];
    V3 sk[R][kMaxReflectDepth];  // surface colours of the reflective levels (unwound innermost first)
    bool act[R], nxt[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      ro[r] = O[r];
      rd[r] = D[r];
      act[r] = inimg[r];
    }
    for (int depth = 0;; ++depth) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        need[r] = false;
        nxt[r] = false;
        sd[r] = v3(0.0f, 0.0f, 1.0f);
        if (!act[r]) continue;
        V3 term;
        if (!found[r]) {
          term = miss_color(fp, py[r]);
        } else {
          const HitInstance ir = load_hit_instance(sc, hit[r].inst);
          P[r] = add(ro[r], muls(rd[r], hit[r].t));
          if (ir.hit_group == 2u) {
            const LightRec& L0 = fp.lights[0];
            ldir[r] = normalize_x<true>(sub(v3(L0.position[0], L0.position[1], L0.position[2]), P[r]));
            nf[r] = face_world_normal<true>(ir, hit[r].prim);
            need[r] = true;
            sd[r] = normalize_x<true>(ldir[r]);
            if (STATS) ++cnt.shadow;
            continue;
          }
          const V3 n = interpolated_world_normal<true>(ir, hit[r].prim, hit[r].u, hit[r].v);
          const V3 s = surface_ref(fp, P[r], n, ro[r]);
          if (MODE == 0 && reflective(fp, ir, depth)) {
            sk[r][depth] = s;
            reflection_ray(P[r], n, rd[r], ro[r], rd[r]);
            nxt[r] = true;
            if (STATS) ++cnt.refl;
            continue;
          }
          term = s;
        }
        // a lane ending its chain at this level holds exactly `depth` reflective levels
        color[r] = unwind_chain(sk[r], depth, term, refl);
        act[r] = false;
      }
      trace_packet<true, STATS, R>(sc, P, sd, 0.01f, 100000.0f, need, occl, sh, cnt);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (!need[r]) continue;
        bool shadowed = dot(nf[r], ldir[r]) < 0.0f;
        if (!shadowed) shadowed = occl[r];
        const float factor = shadowed ? 0.3f : 1.0f;
        const float li = maxf(0.0f, dot(nf[r], ldir[r]));
        const float c = (1.0f * li) * factor;
        const V3 term = v3(c, c, c);
        color[r] = unwind_chain(sk[r], depth, term, refl);
        act[r] = false;
      }
      // uniform exit: no ray of the packet reflects further
      bool more = false;
#pragma unroll
      for (int r = 0; r < R; ++r) more = more || wave_ballot(nxt[r]) != 0;
      if (!more) return;
#pragma unroll
      for (int r = 0; r < R; ++r) act[r] = nxt[r];
      trace_packet<false, STATS, R, true>(sc, ro, rd, 0.001f, 1000.0f, act, found, hit, cnt);
    }
  }
  // RT_SHADE_LAMBERT_SHADOW (MODE 1) and RT_SHADE_PRIMARY (MODE 2)
  V3 n[R];
  float c[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    n[r] = v3(0.0f, 0.0f, 0.0f);
    c[r] = 0.0f;
    if (found[r]) {
      const HitInstance ir = load_hit_instance(sc, hit[r].inst);
      n[r] = ir.hit_group == 2u ? face_world_normal(ir, hit[r].prim)
                                : neg(interpolated_world_normal(ir, hit[r].prim, hit[r].u, hit[r].v));
    }
  }
  for (uint32_t l = 0; l < fp.nlights; ++l) {
    const LightRec& Lr = fp.lights[l];
    float nl[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const V3 L = normalize(sub(v3(Lr.position[0], Lr.position[1], Lr.position[2]), P[r]));
      nl[r] = dot(n[r], L);
      need[r] = found[r] && nl[r] > 0.0f;
      sd[r] = normalize(L);
      occl[r] = false;
      if (MODE == 1 && STATS && need[r]) ++cnt.shadow;
    }
    if (MODE == 1) {
      if (RT_SHADOW_COMPACT && R == 1)
        occl[0] = shadow_compact<STATS>(sc, P[0], sd[0], need[0], l & 1u, cnt);
      else
        trace_packet<true, STATS, R>(sc, P, sd, 0.01f, 100000.0f, need, occl, sh, cnt);
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (need[r]) c[r] = c[r] + nl[r] * (occl[r] ? 0.3f : 1.0f);
  }
  // the miss colour is formed here, not kept live across the shadow walks
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const float v = c[r] / (float)fp.nlights;
    color[r] = found[r] ? v3(v, v, v) : miss_color(fp, py[r]);
  }
}

// The pixel store (RayGen.hlsl:42, gOutput = float4(color, 1) into the R8G8B8A8_UNORM UAV): frame `frame` of
// the launch, RGBA8 or, for the tiled-frame loop's strips, RGB8 (the alpha byte is the constant 255: the assembly
// restores it, so it never crosses xGMI). out_bpp is uniform: one branch per wave. MF false (a launch of one
// RGBA8 frame, rt_dispatch_rays): the plain RGBA8 store, no frame offset and no out_bpp read.
template <bool MF = true>
__device__ __forceinline__ void store_pixel(const FrameParams& fp, uint32_t* out, uint32_t o, V3 a, uint32_t frame) {
  const uint32_t r = unorm8(a.x), g = unorm8(a.y), b = unorm8(a.z);
  if (!MF) {
    out[o] = r | (g << 8) | (b << 16) | (255u << 24);
    return;
  }
  char* base = (char*)out + (size_t)frame * fp.frame_bytes;
  if (fp.out_bpp == 3u) {
    uint8_t* p = (uint8_t*)base + (size_t)o * 3u;
    p[0] = (uint8_t)r;
    p[1] = (uint8_t)g;
    p[2] = (uint8_t)b;
  } else {
    ((uint32_t*)base)[o] = r | (g << 8) | (b << 16) | (255u << 24);
  }
}

// WAVE_FETCH: the fetch counters are wave-uniform (packet schedule) and count once per wave.
template <bool WAVE_FETCH>
__device__ __forceinline__ void flush_stats(const Counters& c, unsigned long long* stats) {
  uint32_t v[12] = {c.primary, c.shadow, c.aabb, c.tri, c.inst, c.overflow, c.refl, c.nfetch, c.tfetch, c.ifetch,
                    c.lnfetch, c.ltfetch};
  const int slot[12] = {0, 1, 2, 3, 4, 5, 8, 9, 10, 11, 9, 10};
  for (int k = 0; k < 12; ++k) {
    unsigned long long x = v[k];
    if (!WAVE_FETCH || k < 7 || k >= 10)
      for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, 64);
    if ((threadIdx.x & 63) == 0 && x) atomicAdd(stats + slot[k], x);
  }
}

#ifdef RT_TRACE_MIN_WAVES
#define RT_TRACE_ATTR __attribute__((amdgpu_waves_per_eu(RT_TRACE_MIN_WAVES, 8)))
#else
#define RT_TRACE_ATTR
#endif

template <int MODE, bool STATS>
__global__ __launch_bounds__(kBlock) RT_TRACE_ATTR void k_trace_frame(SceneView sc, FrameParams fp,
                                                        const uint32_t* __restrict__ rows,
                                                        uint32_t* __restrict__ rgba8,
                                                        float4* __restrict__ rgba32f,
                                                        unsigned long long* __restrict__ stats) {
  extern __shared__ int s_stack[];
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint32_t px = blockIdx.x * 16u + (w & 1u) * 8u + (lane & 7u);
  const uint32_t orow = blockIdx.y * 16u + (w >> 1) * 8u + (lane >> 3);
  Counters cnt;
  if (px < fp.width && orow < fp.nrows) {
    const uint32_t py = rows ? rows[orow] : orow;
    const LaneStack stk =
        lane_stack(sc, s_stack, ((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * kBlock + threadIdx.x);
    const uint32_t k = fp.spp_side;
    V3 acc = v3(0.0f, 0.0f, 0.0f);
    for (uint32_t sy = 0; sy < k; ++sy)
      for (uint32_t sx = 0; sx < k; ++sx) {
        const float ox = ((float)sx + 0.5f) / (float)k;
        const float oy = ((float)sy + 0.5f) / (float)k;
        acc = add(acc, shade_sample<MODE, STATS>(sc, fp, fp.cam[blockIdx.z], px, py, ox, oy, stk, cnt));
      }
    if (k > 1) {
      const float ns = (float)(k * k);
      acc = v3(acc.x / ns, acc.y / ns, acc.z / ns);
    }
    const size_t o = (size_t)orow * fp.width + px;
    store_pixel(fp, rgba8, (uint32_t)o, acc, blockIdx.z);
    if (rgba32f) rgba32f[o] = make_float4(acc.x, acc.y, acc.z, 1.0f);
  }
  if (STATS) flush_stats<false>(cnt, stats);
}

// Wave-packet frame kernel. KS = 1: a wave covers an 8 x 8R pixel tile (ray r of lane l: column
// l % 8, row entry 8r + l / 8 of the tile), one camera sample per pixel. KS = 2 / 4 (spp 4 / 16,
// R = 1): the KS x KS samples of a pixel sit in consecutive lanes and a wave covers an
// (8 / KS) x (8 / KS) pixel tile: every lane traces ONE sample (no accumulator lives across the
// traces, so the multi-sample kernel has the one-sample kernel's registers), the packet's
// footprint on screen shrinks with the sample count (more coherent packets), and the pixel's
// samples are summed across lanes in sample order at the end — the same float additions, in the
// same order, as the sample loop. KS = 0: the sample loop (spp 9, or R > 1). A workgroup is
// RT_PACKET_WX x RT_PACKET_WY waves (2 x 1: 128 threads; multi-sample kernels 1 x 1; smaller workgroups shorten the tail of
// the launch). Rays outside the image or the row list join the packets dead; only in-image
// pixels are stored.
// Occupancy: LAMBERT_SHADOW (the perf configs) runs at 7 waves per SIMD (72 VGPRs, no spills);
// 6 and 8 measured slower overall. REF and PRIMARY keep the allocator's choice (REF would spill
// hundreds of bytes; PRIMARY measured neutral).
#ifndef RT_LS_WAVES
#define RT_LS_WAVES 7
#endif
#ifndef RT_SPP_WAVES
#define RT_SPP_WAVES 4  // the sample-loop kernel (KS = 0, e.g. spp 9) needs 97 VGPRs: 4 waves spill nothing
#endif
#ifndef RT_KS_WAVES
#define RT_KS_WAVES RT_LS_WAVES  // the sample-lane kernels (KS = 2, 4)
#endif
#ifndef RT_REF_WAVES
#define RT_REF_WAVES 1  // REF (MODE 0) one-sample kernel: 1 = the allocator's choice
#endif
#ifndef RT_PACKET_WX
#define RT_PACKET_WX 2  // waves of a packet workgroup along x
#endif
#ifndef RT_PACKET_WY
#define RT_PACKET_WY 1  // ... and along y; 2 x 1 measured best (C4/C5 -6 % vs 2 x 2)
#endif
#ifndef RT_SAMPLE_LANES
#define RT_SAMPLE_LANES 1  // 0: every multi-sample frame uses the sample loop (A/B knob)
#endif
#ifndef RT_PACKET_WX_MS
#define RT_PACKET_WX_MS 1  // multi-sample kernels (KS = 2, 4): one-wave workgroups (C5 -2.8 % vs 2 x 1)
#endif
#ifndef RT_BALANCE_FRONT_PRIO
#define RT_BALANCE_FRONT_PRIO 3  // s_setprio of a work list's front-class waves (0 .. 3)
#endif
#ifndef RT_MS_WIDE
#define RT_MS_WIDE 0  // multi-sample waves: 1 = pixel tiles 8 (or 64 / samples) wide (32-B row stores), 0 = square
#endif
// pixel tile of one wave: 8 x 8 for one sample per pixel; with KS x KS samples per pixel in consecutive lanes
// 64 / KS^2 pixels, square ((8 / KS) x (8 / KS)) or wide (RT_MS_WIDE: 8 x 2 at KS = 2)
__host__ __device__ constexpr uint32_t ms_tile_w(int ks) {
  return ks > 1 ? (RT_MS_WIDE ? (64u / (uint32_t)(ks * ks) < 8u ? 64u / (uint32_t)(ks * ks) : 8u) : 8u / (uint32_t)ks)
                : 8u;
}
__host__ __device__ constexpr uint32_t ms_tile_h(int ks) {
  return ks > 1 ? (64u / (uint32_t)(ks * ks)) / ms_tile_w(ks) : 8u;
}
// waves along x / y of a packet workgroup for the sample layout KS
__host__ __device__ constexpr int packet_wx(int ks) { return ks > 1 ? RT_PACKET_WX_MS : RT_PACKET_WX; }
__host__ __device__ constexpr int packet_wy(int ks) { return ks > 1 ? 1 : RT_PACKET_WY; }
__host__ __device__ constexpr int packet_block(int ks) { return 64 * packet_wx(ks) * packet_wy(ks); }
static_assert(packet_block(1) <= 64 * kMaxPacketWaves && packet_block(2) <= 64 * kMaxPacketWaves,
              "lane_subtree's LDS stacks: one per wave of a packet workgroup");

// BAL: the launch runs a tile-balance work list or records the waves' times (FrameParams::plan / cost); the plain
// grid's kernel carries none of it (a 64-bit start time and the slot live across the whole walk cost registers).
// MF: several frames per launch (grid z / the item's frame: a camera per frame) or RGB8 strips (rt_render_strips);
// false for one RGBA8 frame (rt_dispatch_rays, the bench's frames loop): camera 0 at its fixed kernel-argument
// offset and the plain store, without the per-frame address arithmetic and its dependent argument loads
#ifndef RT_PACKET_HW_WAVES
#define RT_PACKET_HW_WAVES (RT_PACKET_SGPRS && RT_PACKET_SGPRS <= 80 ? 8 : 7)  // resident waves per SIMD (SGPRs)
#endif
#ifndef RT_PACKET_SGPRS
#define RT_PACKET_SGPRS 0  // > 0: cap the packet kernels' SGPRs (amdgpu_num_sgpr), A/B of the hardware residency
#endif
#ifndef RT_PLAIN_SGPRS
// the kernels without the tile balance (the frames loop, the strips, REF): 80 SGPRs (72 used) fit 8 waves per SIMD
// where 84 hold them to 7; the few SGPRs spilled to VGPR lanes cost less than the eighth wave gains since their
// uniform regions stopped being structurized (C2 -1.3 %, C5 -3.7 %, REF -1 %; the balance's kernels lose with the
// cap: C2F +3.5 % one at a time, so they keep theirs)
#define RT_PLAIN_SGPRS 80
#endif
#if RT_PACKET_SGPRS
#define RT_PACKET_SGPR_ATTR __attribute__((amdgpu_num_sgpr(RT_PACKET_SGPRS)))
#else
#define RT_PACKET_SGPR_ATTR
#endif
// The frame kernel, defined twice from rt_trace_packet.inc (amdgpu_num_sgpr takes no template-dependent value):
// k_trace_frame_packet8, held to RT_PLAIN_SGPRS so that it fits 8 waves per SIMD, for the launches that can use the
// eighth wave — no tile balance, no counters, a one-sample tile layout (KS >= 1: <= 64 VGPRs) and not the reflective
// REF kernel (MODE 0: 84 VGPRs); k_trace_frame_packet, with the compiler's own budget, for every other launch.
#if RT_PACKET_SGPRS
#define RT_PLAIN_SGPR_ATTR RT_PACKET_SGPR_ATTR
#elif RT_PLAIN_SGPRS
#define RT_PLAIN_SGPR_ATTR __attribute__((amdgpu_num_sgpr(RT_PLAIN_SGPRS)))
#else
#define RT_PLAIN_SGPR_ATTR
#endif
#define RT_PK_NAME k_trace_frame_packet8
#define RT_PK_SGPR_ATTR RT_PLAIN_SGPR_ATTR
#include "rt_trace_packet.inc"
#undef RT_PK_NAME
#undef RT_PK_SGPR_ATTR
#define RT_PK_NAME k_trace_frame_packet
#define RT_PK_SGPR_ATTR RT_PACKET_SGPR_ATTR
#include "rt_trace_packet.inc"
#undef RT_PK_NAME
#undef RT_PK_SGPR_ATTR


template <bool ANY_HIT, bool STATS, bool CULL>
__global__ __launch_bounds__(kBlock) void k_trace_rays(SceneView sc, const float4* __restrict__ rays,
                                                       uint32_t n, uint4* __restrict__ hits,
                                                       float2* __restrict__ uv,
                                                       unsigned long long* __restrict__ stats) {
  extern __shared__ int s_stack[];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  Counters cnt;
  if (i < n) {
    const float4 a = rays[2 * i], b = rays[2 * i + 1];
    HitRec h;
    const bool f = trace<ANY_HIT, STATS, CULL>(sc, v3(a.x, a.y, a.z), v3(b.x, b.y, b.z), a.w, b.w, h,
                                         lane_stack(sc, s_stack, i), cnt);
    if (STATS) ++cnt.primary;
    hits[i] = make_uint4(__float_as_uint(f ? h.t : b.w), f ? h.inst : 0xffffffffu,
                         f ? h.prim : 0xffffffffu, f ? 1u : 0u);
    if (uv) uv[i] = make_float2(f ? h.u : 0.0f, f ? h.v : 0.0f);
  }
  if (STATS) flush_stats<false>(cnt, stats);
}

// Un-interleaves the gathered strips (rank-major blocks; rank k holds strips s % nranks == k) into the RGBA8 frame.
// in_bpp 3: the strips are RGB8 and the constant alpha 255 is restored here (RayGen.hlsl:42 writes float4(c, 1)).
__global__ void k_assemble(uint32_t W, uint32_t H, uint32_t nranks, uint32_t strip_rows,
                           const uint8_t* __restrict__ in, uint32_t* __restrict__ out,
                           uint32_t rows_per_rank, uint32_t in_bpp) {
  // one thread per output pixel (4 B), coalesced along x
  const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t y = blockIdx.y;
  if (x >= W || y >= H) return;
  const uint32_t s = y / strip_rows, within = y % strip_rows;
  const uint32_t rank = s % nranks, local_strip = s / nranks;
  const uint32_t lrow = local_strip * strip_rows + within;
  const size_t src = ((size_t)rank * rows_per_rank + lrow) * W + x;
  uint32_t v;
  if (in_bpp == 3u) {
    const uint8_t* p = in + src * 3u;
    v = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | (255u << 24);
  } else {
    v = ((const uint32_t*)in)[src];
  }
  out[(size_t)y * W + x] = v;
}

// 16 B per thread (W % 4 == 0, 16-B aligned buffers): kAsmRows output rows per workgroup, so the
// copy is few short waves that interleave with a concurrent frame's trace waves instead of
// flooding the dispatcher (one 4-B thread per pixel is 8 K workgroups per 1080p frame)
constexpr uint32_t kAsmRows = 8;
__global__ __launch_bounds__(256) void k_assemble16(uint32_t W4, uint32_t H, uint32_t nranks, uint32_t strip_rows,
                                                    const uint4* __restrict__ in, uint4* __restrict__ out,
                                                    uint32_t rows_per_rank) {
  const uint32_t x = blockIdx.x * 256u + threadIdx.x;
  if (x >= W4) return;
  const uint32_t y0 = blockIdx.y * kAsmRows;
#pragma unroll
  for (uint32_t i = 0; i < kAsmRows; ++i) {
    const uint32_t y = y0 + i;
    if (y >= H) break;
    const uint32_t s = y / strip_rows, within = y % strip_rows;
    const uint32_t rank = s % nranks, local_strip = s / nranks;
    const uint32_t lrow = local_strip * strip_rows + within;
    out[(size_t)y * W4 + x] = in[((size_t)rank * rows_per_rank + lrow) * W4 + x];
  }
}

// The same from RGB8 strips: 4 pixels = 12 B (three dwords, 4-B aligned: a strip row is 3 W bytes with W % 4 == 0)
// in, 16 B out with the alpha bytes set. Dwords a, b, c hold r0 g0 b0 r1 | g1 b1 r2 g2 | b2 r3 g3 b3. The frames of
// a batched gather in one launch (grid z = frame b: its strips frame_words x b words into every rank's block).
struct AsmFrames {
  uint4* out[kMaxLaunchFrames];
};
// 3 words of RGB8 (4 pixels) -> 4 RGBA8 words, alpha 255
__device__ __forceinline__ uint4 rgb4_to_rgba(uint32_t a, uint32_t b, uint32_t c) {
  return make_uint4((a & 0xffffffu) | 0xff000000u, (a >> 24) | ((b & 0xffffu) << 8) | 0xff000000u,
                    (b >> 16) | ((c & 0xffu) << 16) | 0xff000000u, (c >> 8) | 0xff000000u);
}
// The strips of rt_comm into RGBA8 frames, 16 pixels per thread (W % 16 == 0, 16-B aligned buffers): three 16-B
// loads and four 16-B stores per thread, consecutive lanes on consecutive 48-B / 64-B chunks of one row (a wave
// reads 3 KB and writes 4 KB contiguously); one thread per (row, 16-pixel group) of every frame of the batch (z).
__global__ __launch_bounds__(256) void k_assemble48_rgb(uint32_t W16, uint32_t H, uint32_t nranks, uint32_t strip_rows,
                                                        const uint4* __restrict__ in_all, AsmFrames outs,
                                                        uint32_t rows_per_rank, uint32_t frame_vec4) {
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  if (t >= W16 * H) return;
  const uint32_t y = t / W16, xg = t - y * W16;
  const uint32_t s = y / strip_rows, within = y % strip_rows;
  const uint32_t rank = s % nranks, local_strip = s / nranks;
  const uint32_t lrow = local_strip * strip_rows + within;
  const uint4* p = in_all + (size_t)blockIdx.z * frame_vec4 + ((size_t)rank * rows_per_rank + lrow) * (W16 * 3u) + xg * 3u;
  const uint4 q0 = p[0], q1 = p[1], q2 = p[2];
  uint4* o = outs.out[blockIdx.z] + (size_t)y * (W16 * 4u) + xg * 4u;
  o[0] = rgb4_to_rgba(q0.x, q0.y, q0.z);
  o[1] = rgb4_to_rgba(q0.w, q1.x, q1.y);
  o[2] = rgb4_to_rgba(q1.z, q1.w, q2.x);
  o[3] = rgb4_to_rgba(q2.y, q2.z, q2.w);
}
__global__ __launch_bounds__(256) void k_assemble16_rgb(uint32_t W4, uint32_t H, uint32_t nranks, uint32_t strip_rows,
                                                        const uint32_t* __restrict__ in_all, AsmFrames outs,
                                                        uint32_t rows_per_rank, uint32_t frame_words) {
  const uint32_t x = blockIdx.x * 256u + threadIdx.x;
  if (x >= W4) return;
  const uint32_t* in = in_all + (size_t)blockIdx.z * frame_words;
  uint4* out = outs.out[blockIdx.z];
  const uint32_t y0 = blockIdx.y * kAsmRows;
#pragma unroll
  for (uint32_t i = 0; i < kAsmRows; ++i) {
    const uint32_t y = y0 + i;
    if (y >= H) break;
    const uint32_t s = y / strip_rows, within = y % strip_rows;
    const uint32_t rank = s % nranks, local_strip = s / nranks;
    const uint32_t lrow = local_strip * strip_rows + within;
    const uint32_t* p = in + (((size_t)rank * rows_per_rank + lrow) * W4 + x) * 3u;
    const uint32_t a = p[0], b = p[1], c = p[2];
    out[(size_t)y * W4 + x] = make_uint4((a & 0xffffffu) | 0xff000000u, (a >> 24) | ((b & 0xffffu) << 8) | 0xff000000u,
                                         (b >> 16) | ((c & 0xffu) << 16) | 0xff000000u, (c >> 8) | 0xff000000u);
  }
}

// whether a launch needs the general frame kernel (MF): several frames, or RGB8 strips
__host__ inline bool launch_multi_frame(const FrameParams& fp) { return fp.nframes > 1u || fp.out_bpp != 4u; }

template <int MODE, bool STATS>
hipError_t launch_mode(const SceneView& sc, const FrameParams& fp, const uint32_t* rows, void* rgba8,
                       float* rgba32f, unsigned long long* stats, int schedule, uint32_t plan_items, hipStream_t s) {
  dim3 grid((fp.width + 15) / 16, (fp.nrows + 15) / 16, fp.nframes);
  const PacketGeometry g = packet_geometry(sc, fp, schedule);
  if (g.packet) {
    constexpr int R = RT_PACKET_RAYS;
    const int ks = g.ks;
    // the plain grid, or (tile balance) one wave per work-list item, as many as the list's budget
    dim3 gp = fp.plan ? dim3((plan_items + g.wl - 1) / g.wl) : dim3(g.grid_x, g.grid_y, fp.nframes);
    // counter passes always take the general (MF) kernel: fewer instantiations
    const bool mf = STATS || launch_multi_frame(fp);
#define RT_LAUNCH_PACKET_K(KS, BALV, MFV)                                                                      \
  do {                                                                                                         \
    if constexpr (!BALV && !STATS && MODE != 0 && (R == 1 ? KS : 0) >= 1)                                        \
      hipLaunchKernelGGL((k_trace_frame_packet8<MODE, STATS, R, (R == 1 ? KS : 0), BALV, MFV>), gp,           \
                         dim3(packet_block(R == 1 ? KS : 0)), 0, s, sc, fp, rows, (uint32_t*)rgba8,             \
                         (float4*)rgba32f, stats);                                                             \
    else                                                                                                       \
      hipLaunchKernelGGL((k_trace_frame_packet<MODE, STATS, R, (R == 1 ? KS : 0), BALV, MFV>), gp,            \
                         dim3(packet_block(R == 1 ? KS : 0)), 0, s, sc, fp, rows, (uint32_t*)rgba8,             \
                         (float4*)rgba32f, stats);                                                             \
  } while (0)
#define RT_LAUNCH_PACKET(KS)                                                                                   \
  do {                                                                                                         \
    if constexpr (STATS) {                                                                                     \
      if (fp.plan || fp.cost) RT_LAUNCH_PACKET_K(KS, true, true);                                              \
      else RT_LAUNCH_PACKET_K(KS, false, true);                                                                \
    } else if (fp.plan || fp.cost) {                                                                           \
      if (mf) RT_LAUNCH_PACKET_K(KS, true, true);                                                              \
      else RT_LAUNCH_PACKET_K(KS, true, false);                                                                \
    } else {                                                                                                   \
      if (mf) RT_LAUNCH_PACKET_K(KS, false, true);                                                             \
      else RT_LAUNCH_PACKET_K(KS, false, false);                                                               \
    }                                                                                                          \
  } while (0)
    if (ks == 1) RT_LAUNCH_PACKET(1);
    else if (ks == 2) RT_LAUNCH_PACKET(2);
    else if (ks == 4) RT_LAUNCH_PACKET(4);
    else RT_LAUNCH_PACKET(0);
#undef RT_LAUNCH_PACKET
#undef RT_LAUNCH_PACKET_K
  } else {
    size_t lds = (size_t)sc.lds_cap * kBlock * sizeof(int);
    hipLaunchKernelGGL((k_trace_frame<MODE, STATS>), grid, dim3(kBlock), lds, s, sc, fp, rows,
                       (uint32_t*)rgba8, (float4*)rgba32f, stats);
  }
  return hipGetLastError();
}

}  // namespace

PacketGeometry packet_geometry(const SceneView& sc, const FrameParams& fp, int schedule) {
  PacketGeometry g;
  g.packet = schedule == RT_SCHED_PACKET && sc.packet_cap < kPacketStack;
  if (!g.packet) return g;
  constexpr int R = RT_PACKET_RAYS;
  // KS: 1 one sample per pixel; 2 / 4 the k x k samples of a pixel in consecutive lanes; 0 the loop
  g.ks = fp.spp_side == 1 ? 1 : ((RT_SAMPLE_LANES && R == 1 && (fp.spp_side == 2 || fp.spp_side == 4))
                                     ? (int)fp.spp_side : 0);
  const uint32_t tp = ms_tile_w(g.ks);
  const uint32_t tr = (g.ks <= 1 && fp.tile_rows == 4u) ? 4u : ms_tile_h(g.ks);  // as the kernel's TR
  g.wx = (uint32_t)packet_wx(g.ks);
  g.wy = (uint32_t)packet_wy(g.ks);
  g.wl = g.wx * g.wy;
  const uint32_t tw = tp * g.wx, th = tr * R * g.wy;
  g.grid_x = (fp.width + tw - 1) / tw;
  g.grid_y = (fp.nrows + th - 1) / th;
  g.waves_per_frame = g.grid_x * g.grid_y * g.wl;
  // a tile splits into 2 x 2 parts when both sides are >= 2 pixels, 4 x 4 when >= 4 (one ray per lane only)
  const uint32_t side = tp < tr ? tp : tr;
  g.kmax_code = (R != 1 || RT_SHADOW_COMPACT) ? 0u : side >= 8u ? 3u : side >= 4u ? 2u : side >= 2u ? 1u : 0u;
  // the shadow-ray compaction variant synchronises a workgroup's waves (barriers): no work list there, whose waves
  // past its end exit early
  g.plannable = !RT_SHADOW_COMPACT;
  return g;
}

hipError_t launch_trace_frame(const SceneView& sc, const FrameParams& fp, const uint32_t* d_rows,
                              void* rgba8, float* rgba32f, unsigned long long* d_stats, bool stats,
                              int schedule, uint32_t plan_items, hipStream_t s) {
  switch (fp.shade_mode) {
    case 0:
      // the reference scene's parity config pins reflectivity to 0: a kernel without
      // the reflection-chain state (registers, the per-lane sk[] stack) then runs at a higher occupancy
      if (fp.material.reflectivity == 0.0f && RT_REF_NOREFL)
        return stats ? launch_mode<3, true>(sc, fp, d_rows, rgba8, rgba32f, d_stats, schedule, plan_items, s)
                     : launch_mode<3, false>(sc, fp, d_rows, rgba8, rgba32f, d_stats, schedule, plan_items, s);
      return stats ? launch_mode<0, true>(sc, fp, d_rows, rgba8, rgba32f, d_stats, schedule, plan_items, s)
                   : launch_mode<0, false>(sc, fp, d_rows, rgba8, rgba32f, d_stats, schedule, plan_items, s);
    case 1:
      return stats ? launch_mode<1, true>(sc, fp, d_rows, rgba8, rgba32f, d_stats, schedule, plan_items, s)
                   : launch_mode<1, false>(sc, fp, d_rows, rgba8, rgba32f, d_stats, schedule, plan_items, s);
    case 2:
      return stats ? launch_mode<2, true>(sc, fp, d_rows, rgba8, rgba32f, d_stats, schedule, plan_items, s)
                   : launch_mode<2, false>(sc, fp, d_rows, rgba8, rgba32f, d_stats, schedule, plan_items, s);
    default:
      return hipErrorInvalidValue;
  }
}

// ------------------------------------------------------------------------------------------
// Tile balance: the wave work list of one launch (k_tile_plan, one workgroup). A frame lasts as long as its
// slowest tiles (a wave walks the union of its 64 rays' paths; on C4 one 8 x 8 tile takes as long as the rest of
// the frame, profiles/r03_wave_times_C4.txt). The packet kernel leaves two words per tile (FrameParams::cost): the
// time of its last whole wave (w), and the costliest part of its last split (p, time << 2 | layout). From them:
// the load bound L = sum(w) / the GPU's wave slots. The plan pays only while the costliest tile outlasts L (it
// then forms the launch's tail); otherwise the list is the plain grid's order. When it pays, T = max(L, 0.35 x the
// costliest tile): a tile above T is traced as 4 parts (2 x 2 sub-rectangles) when 0.55 x its time fits T, else
// as 16 — unless its last split measured a part above 0.8 x the whole (coherent rays: the parts walk nearly the
// whole tile's nodes each, so splitting only adds waves), which keeps it whole. The items are then laid out in two
// classes, those estimated above a fraction of L first, each class in tile order: the long waves start at the
// front, and neighbouring waves still trace neighbouring tiles (they share the BVH nodes in the scalar cache and
// L2; a strict longest-first order scattered them and lost more than the tail it saved, profiles/
// r04_balance_ab_v1.txt). The list is always a valid cover (each tile once, or each of its parts once) whatever
// the costs hold: the image never depends on it, only the schedule. Items beyond the grid's budget are refused by
// raising T. (tools/split_study.py models the split on the oracle's packet fetches.) The north star's "wavefront
// ballot/prefix-sum" appears here as the block scan that places each item.
// ------------------------------------------------------------------------------------------
#ifndef RT_PLAN_THREADS
#define RT_PLAN_THREADS 1024  // the plan workgroup (A/B: 512 needs 2 free wave slots per SIMD to dispatch, not 4)
#endif
#ifndef RT_PLAN_PRIO
#define RT_PLAN_PRIO 0  // s_setprio of the plan's waves (A/B: issue ahead of the trace waves sharing their SIMDs)
#endif
constexpr uint32_t kPlanThreads = RT_PLAN_THREADS;
static_assert(kPlanMaxTiles <= 64u * kPlanThreads, "a run of at most 64 tiles per thread (sums of 16-bit times)");

// exclusive prefix sum over the workgroup (wave scan by shuffles, the waves' totals through LDS)
__device__ __forceinline__ uint64_t block_excl_scan64(uint64_t v, uint64_t* s_w, uint64_t* total) {
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  uint64_t x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  __syncthreads();  // s_w may still be read by the previous reduction
  if (lane == 63u) s_w[wv] = x;
  __syncthreads();
  uint64_t before = 0, tot = 0;
  for (uint32_t k = 0; k < kPlanThreads / 64u; ++k) {
    const uint64_t s = s_w[k];
    before += k < wv ? s : 0u;
    tot += s;
  }
  *total = tot;
  return before + x - v;
}

// forced layouts (tests: the oracle emulates the same parts): 1 every tile in 4, 2 every tile in 16, 3 by tile
// position ((tx + 2 ty) % 3: whole, 4, 16), 4 every tile in 64 (one pixel each), capped by the tile shape
__device__ __forceinline__ uint32_t plan_forced(const PlanArgs& a, uint32_t t) {
  uint32_t code = a.force == 1u ? 1u : a.force == 2u ? 2u : a.force == 4u ? 3u : 0u;
  if (a.force == 3u) {
    const uint32_t f = t % a.waves_per_frame, wg = f / a.wl, w = f % a.wl;
    const uint32_t tx = (wg % a.grid_x) * a.wx + w % a.wx, ty = (wg / a.grid_x) * a.wy + w / a.wx;
    code = (tx + 2u * ty) % 3u;
  }
  return code < a.kmax_code ? code : a.kmax_code;
}

__device__ uint64_t block_sum64(uint64_t v, uint64_t* sh) {
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63u) == 0u) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t t = 0;
  for (uint32_t k = 0; k < kPlanThreads / 64u; ++k) t += sh[k];
  return t;
}

__device__ uint64_t block_max64(uint64_t v, uint64_t* sh) {
  for (int o = 32; o >= 1; o >>= 1) {
    const uint64_t q = __shfl_xor(v, o, 64);
    v = q > v ? q : v;
  }
  __syncthreads();
  if ((threadIdx.x & 63u) == 0u) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t m = 0;
  for (uint32_t k = 0; k < kPlanThreads / 64u; ++k) m = sh[k] > m ? sh[k] : m;
  return m;
}

// One workgroup. The launch's snapshot of the costs lives in LDS (launches of the same shape on other streams write
// the costs meanwhile, and every step must see the same values): one word per tile — the whole wave's time in bits
// 0..15 (10-ns ticks up to 655 us), the last split's costliest part in bits 16..30 (80-ns units in 13 bits, its
// layout in 2) and bit 31, "parts ran since the whole time" — at a padded index (a word per 32 tiles) so a thread's
// run of consecutive tiles is bank-conflict free. No pass goes back to memory: thread i owns tiles [m i, m i + m)
// (m = ceil(ntiles / 1024)); one block scan places every thread's items (front class, then the rest, each in tile
// order).
__device__ __forceinline__ uint32_t plan_lds_ix(uint32_t t) { return t + (t >> 5); }

__device__ __forceinline__ uint32_t plan_pack(uint32_t w, uint32_t p) {
  const uint32_t wt = w & 0x7fffffffu;
  const uint32_t w16 = wt < 0xffffu ? wt : 0xffffu;
  const uint32_t pt = (p >> 2) >> 3;  // the part's time in 80-ns units
  const uint32_t p15 = p ? ((pt < 0x1fffu ? pt : 0x1fffu) << 2) | (p & 3u) : 0u;
  return w16 | (p15 << 16) | (w & 0x80000000u);
}

// A tile's current cost: its last whole wave's time, or — when parts of a split ran since (the whole time is then
// older than them) — the whole estimated from its costliest part (the inverse of the part estimates in
// plan_pick32: 0.55 / 0.35 / 0.21 of the whole). So a split tile whose view became cheap is seen cheap, is traced
// whole again and measures a fresh whole time; a stale whole time never keeps it split.
// x 20 / 11, 20 / 7 and 1 / 0.21 in 10-bit fixed point
__device__ __forceinline__ uint32_t plan_inv_part(uint32_t code) { return code == 1u ? 1862u : code == 2u ? 2926u : 4876u; }
__device__ __forceinline__ uint32_t plan_cur(uint32_t c) {
  const uint32_t w = c & 0xffffu, p15 = (c >> 16) & 0x7fffu;
  if (!(c >> 31) || !p15) return w;
  const uint32_t pt = (p15 >> 2) << 3, e = (pt * plan_inv_part(p15 & 3u)) >> 10;
  return e < 0xffffu ? e : 0xffffu;
}

// plan_cur from the raw cost words, for the snapshot loop (plan_cur of the packed word there, or one product by a
// selected constant, crashes this compiler's instruction selection: ROCm 7.2 clang 22, AMDGPU DAG->DAG)
__device__ __forceinline__ uint32_t plan_cur_raw(uint32_t w16, uint32_t p, bool since) {
  const uint32_t q = (p >> 5) < 0x1fffu ? (p >> 5) : 0x1fffu;  // the part in 80-ns units, as plan_pack keeps it
  const uint32_t e = (p & 3u) == 1u ? ((q << 3) * 1862u) >> 10
                                    : (p & 3u) == 2u ? ((q << 3) * 2926u) >> 10 : ((q << 3) * 4876u) >> 10;
  return since && p ? (e < 0xffffu ? e : 0xffffu) : w16;
}

// the layout of a tile from its snapshot word and its estimated time; 32-bit: a time is at most 65535 ticks, and T
// (0xffffffff: split nothing) is below 65535 wherever a tile exceeds it
__device__ __forceinline__ uint32_t plan_pick32(const PlanArgs& a, bool split, uint32_t c, uint32_t T, uint32_t* est) {
  const uint32_t w = c & 0xffffu, p15 = (c >> 16) & 0x7fffu, pt = (p15 >> 2) << 3;  // the part's time in ticks
  const uint32_t cur = plan_cur(c);
  uint32_t code = 0;
  // 4 parts when 0.55 x the tile fits T, else 16 when 0.35 x fits (or 4 x 4 is the finest the tile allows), else 64
  // single-pixel parts (the worst C4 tiles' costliest pixel walks 0.2 of the whole packet's fetches,
  // tools/path_study.py)
  if (split && a.kmax_code && cur > T)
    code = (a.kmax_code == 1u || cur * 11u <= T * 20u) ? 1u : (a.kmax_code == 2u || cur * 7u <= T * 20u) ? 2u : 3u;
  // the last split of this tile measured a part above 0.8 x its whole wave: splitting does not pay there
  if (code && p15 && pt * 5u > w * 4u) code = 0u;
  *est = code == 0u ? cur
                    : (p15 && (p15 & 3u) == code) ? pt
                    : (code == 1u ? (cur * 11u) / 20u : code == 2u ? (cur * 7u) / 20u : (cur * 215u) >> 10);
  return code;
}

__global__ __launch_bounds__(kPlanThreads) void k_tile_plan(PlanArgs a) {
  __shared__ uint32_t s_c[kPlanMaxTiles + kPlanMaxTiles / 32];
  __shared__ uint64_t s_red[kPlanThreads / 64];
  if (RT_PLAN_PRIO) __builtin_amdgcn_s_setprio(RT_PLAN_PRIO);
  const uint64_t t_begin = __builtin_amdgcn_s_memrealtime();
  const uint32_t tid = threadIdx.x, n = a.ntiles, cap = n + a.extra_cap;
  const uint32_t G = plan_groups(cap, a.wl);  // the launch's workgroups: the items' storage map (plan_xaddr)
  const uint32_t m = (n + kPlanThreads - 1) / kPlanThreads, t0 = tid * m, t1 = t0 + m < n ? t0 + m : n;
  // 1. the snapshot (coalesced loads, tile t by thread t % 1024, unrolled so the loads overlap) and the load bound
  uint32_t lsum = 0, lmax = 0;  // < 64 tiles x 65535 per thread
  uint32_t lsplits = 0;          // the tiles' measured splits: useless << 16 | useful
  if (!a.force) {
#pragma unroll 8
    for (uint32_t t = tid; t < n; t += kPlanThreads) {
      const uint2 v = reinterpret_cast<const uint2*>(a.cost)[t];
      const uint32_t c = plan_pack(v.x, v.y), wx = v.x & 0x7fffffffu;
      const uint32_t cur = plan_cur_raw(c & 0xffffu, v.y, (v.x >> 31) != 0u);
      s_c[plan_lds_ix(t)] = c;
      lsum += cur;
      lmax = cur > lmax ? cur : lmax;
      if (v.y && wx) lsplits += ((uint64_t)(v.y >> 2) * 5u > (uint64_t)wx * 4u) ? 0x10000u : 1u;
    }
  }
  uint32_t T = 0xffffffffu, mx = 0, L = 0, want = 0;
  uint64_t sum = 0;
  bool tail = false, split = a.split != 0u;
  if (!a.force) {
    sum = block_sum64(lsum, s_red);  // its barriers also publish s_c
    mx = (uint32_t)block_max64(lmax, s_red);
    // the shape's tiles are coherent (every measured split had a part above 0.8 x the whole, and there are enough
    // of them to say so): no splitting at all, instead of learning it a few hundred tiles per plan. One split that
    // paid keeps it on: on C2F most splits are useless, the few that pay carry the share (0.071 -> 0.045 ms).
    const uint64_t sp = block_sum64(((uint64_t)(lsplits >> 16) << 32) | (lsplits & 0xffffu), s_red);
    const uint32_t useless = (uint32_t)(sp >> 32), useful = (uint32_t)sp;
    if (useless >= 16u && useful == 0u) split = false;
    L = (uint32_t)(sum / (a.slots ? a.slots : 1u));
    // the costliest tile outlasts the load bound by a quarter and by more than this kernel takes
    tail = (uint64_t)mx * 4u > (uint64_t)L * 5u && mx > L + a.min_gain;
  }
  const uint64_t t_loaded = __builtin_amdgcn_s_memrealtime();
  if (tail) {
    // the floor a split can reach: the costliest part of the finest split allowed (0.35 of the tile at 16 parts,
    // 0.21 at 64)
    const uint32_t F = a.kmax_code >= 3u ? (mx * 215u) >> 10 : (mx * 7u) / 20u;
    T = L > F ? L : F;
    // 2. the parts must fit the grid's budget: raise T until they do (the first count is the demand, reported)
    for (int iter = 0; split && iter < 24; ++iter) {
      uint32_t ex = 0, e;
#pragma unroll 4
      for (uint32_t t = tid; t < n; t += kPlanThreads)
        ex += split_parts(plan_pick32(a, split, s_c[plan_lds_ix(t)], T, &e)) - 1u;
      const uint64_t tot = block_sum64(ex, s_red);
      if (iter == 0) want = (uint32_t)(tot < 0xffffffffull ? tot : 0xffffffffull);
      if (tot <= a.extra_cap) break;
      T = (iter < 23 && T < 65535u) ? T + T / 4u + 1u : 0xffffffffu;  // the last resort: no tile split
    }
  }
  const uint64_t t_budget = __builtin_amdgcn_s_memrealtime();
  uint32_t nsplit = 0, nitems = n, refused = 0, lref = 0;
  bool pays = false;
  if (!a.force && !tail) {
    // no tail: the plain grid's order, every tile whole
#pragma unroll 4
    for (uint32_t t = tid; t < n; t += kPlanThreads) a.plan[1u + plan_xaddr(t, a.wl, G)] = t << 8;
  } else {
    // 3. each tile's layout and class (estimated above front / 16 x L: first); thread i's run of tiles
    // [m i, m i + m) counts its items, one block scan of the runs' (front, rest) counts places them, and each
    // tile's first item position (with its layout) replaces its snapshot word
    const uint32_t TF = (!a.force && a.front) ? (L * a.front) >> 4 : 0xffffffffu;
    uint32_t cf = 0, cb = 0, tf = 0, e = 0;
#pragma unroll 4
    for (uint32_t t = t0; t < t1; ++t) {
      const uint32_t code = a.force ? plan_forced(a, t) : plan_pick32(a, split, s_c[plan_lds_ix(t)], T, &e);
      const uint32_t k = split_parts(code);
      const bool fr = !a.force && e > TF;
      cf += fr ? k : 0u;
      cb += fr ? 0u : k;
      tf += fr ? 1u : 0u;
      nsplit += code ? 1u : 0u;
    }
    uint64_t tot;
    const uint64_t ex = block_excl_scan64(((uint64_t)cf << 32) | cb, s_red, &tot);
    const uint32_t nfront_items = (uint32_t)(tot >> 32);  // the front class occupies the list's first positions
    uint32_t pf = (uint32_t)(ex >> 32), pb = (uint32_t)(tot >> 32) + (uint32_t)ex;
#pragma unroll 4
    for (uint32_t t = t0; t < t1; ++t) {
      const uint32_t code = a.force ? plan_forced(a, t) : plan_pick32(a, split, s_c[plan_lds_ix(t)], T, &e);
      const uint32_t k = split_parts(code);
      const bool fr = !a.force && e > TF;
      s_c[plan_lds_ix(t)] = ((fr ? pf : pb) << 2) | code;
      if (fr) pf += k;
      else pb += k;
    }
    __syncthreads();
    // 4. the items, tile t by thread t % 1024 again: neighbouring lanes write neighbouring words. An item past the
    // budget is refused and counted (the budget loop above makes that impossible; if it ever happens, the list falls
    // back to the plain grid's below, and PlanStats reports it: VERDICT r4 #6)
#pragma unroll 4
    for (uint32_t t = tid; t < n; t += kPlanThreads) {
      const uint32_t d = s_c[plan_lds_ix(t)], code = d & 3u, k = split_parts(code), pos = d >> 2;
      for (uint32_t q = 0; q < k; ++q) {
        if (pos + q < cap)
          a.plan[1u + plan_xaddr(pos + q, a.wl, G)] =
              (t << 8) | (q << 2) | code | ((a.prio && pos + q < nfront_items) ? 0x80000000u : 0u);
        else ++lref;
      }
      // a split tile's part word restarts (its parts raise it with atomicMax at their end)
      if (!a.force && code) a.cost[2u * t + 1u] = 0u;
    }
    const uint32_t all = (uint32_t)(tot >> 32) + (uint32_t)tot;
    nitems = all < cap ? all : cap;
    // whether the list differs from the plain grid's in what the launch's time depends on: a tile split, or (more
    // waves than the GPU's slots) a front class that is neither empty nor everything
    const uint64_t r = block_sum64(((uint64_t)nsplit << 32) | tf, s_red);
    nsplit = (uint32_t)(r >> 32);
    const uint32_t nfront_tiles = (uint32_t)r;
    pays = nsplit > 0u || (n > a.slots && nfront_tiles > 0u && nfront_tiles < n);
  }
  // its barriers also order every item store before the fallback's
  refused = (uint32_t)block_sum64(lref, s_red);
  if (refused) {
    // a list missing any part would leave pixels unwritten: the plain grid's list instead (every tile whole)
    for (uint32_t t = tid; t < n; t += kPlanThreads) a.plan[1u + plan_xaddr(t, a.wl, G)] = t << 8;
    nitems = n;
    nsplit = 0;
    pays = false;
  }
  const uint64_t t_placed = __builtin_amdgcn_s_memrealtime();
  // diagnostics (PlanArgs::check): the list must cover every tile exactly once — each tile's items one layout, its
  // parts 0 .. k - 1 once each (the words after the items count them: the layouts seen, parts 0 .. 31, parts 32 .. 63)
  uint32_t bad = 0, first_bad = 0xffffffffu, first_word = 0;
  if (a.check) {
    uint32_t* sw = a.plan + 1u + plan_xwords(cap, a.wl);
    uint32_t* sp = sw + n;
    uint32_t* sq = sp + n;
    __syncthreads();  // every item is written
    for (uint32_t t = tid; t < n; t += kPlanThreads) sw[t] = sp[t] = sq[t] = 0u;
    __syncthreads();
    for (uint32_t i = tid; i < nitems; i += kPlanThreads) {
      const uint32_t it = a.plan[1u + plan_xaddr(i, a.wl, G)], slot = (it >> 8) & kPlanSlotMask, q = (it >> 2) & 63u,
                     code = it & 3u;
      if (slot >= n || q >= split_parts(code)) {
        bad += 1u;
        continue;
      }
      atomicAdd(q < 32u ? &sp[slot] : &sq[slot], 1u << (q & 31u));
      atomicOr(&sw[slot], 1u << code);
    }
    __syncthreads();
    for (uint32_t t = tid; t < n; t += kPlanThreads) {
      const uint32_t m = sw[t], c = sp[t], c2 = sq[t];
      const bool ok = (m == 1u && c == 1u && c2 == 0u) || (m == 2u && c == 0xfu && c2 == 0u) ||
                      (m == 4u && c == 0xffffu && c2 == 0u) || (m == 8u && c == 0xffffffffu && c2 == 0xffffffffu);
      if (!ok) {
        bad += 1u;
        if (t < first_bad) {
          first_bad = t;
          first_word = (m << 24) | (c & 0xffffffu);
        }
      }
    }
    bad = (uint32_t)block_sum64(bad, s_red);
    const uint64_t fb = block_max64(~(((uint64_t)first_bad << 32) | first_word), s_red);  // the lowest tile
    first_bad = (uint32_t)(~fb >> 32);
    first_word = (uint32_t)~fb;
  }
  // the item count (the trace waves past it exit), and the summary for the host (host-mapped memory: read at a
  // later dispatch, no copy call)
  if (tid == 0u) {
    a.plan[0] = nitems;
    if (a.stats) {
      PlanStats* st = a.stats;
      st->nitems = nitems;
      st->nsplit = nsplit;
      st->want_extra = want;
      st->max_cost = mx;
      st->mean_cost = n ? (uint32_t)(sum / n) : 0u;
      st->threshold = T;
      st->pays = pays ? 1u : 0u;
      st->coherent = (!a.force && a.split && !split) ? 1u : 0u;
      st->plans += 1u;
      st->refused += refused;
      st->refused_plans += refused ? 1u : 0u;
      st->slots = a.slots;
      // thread 0's view of the phases (10-ns ticks): load + bound, budget, layout + positions + items
      st->phase_ticks[0] = (uint32_t)(t_loaded - t_begin);
      st->phase_ticks[1] = (uint32_t)(t_budget - t_loaded);
      st->phase_ticks[2] = (uint32_t)(t_placed - t_budget);
      if (a.check) {
        st->bad += bad;
        if (bad && !st->first_bad_word) {
          st->first_bad_tile = first_bad;
          st->first_bad_word = first_word | 0x80000000u;
        }
      }
    }
  }
}

namespace {
template <int MODE, int KS>
const void* bal_kernel(bool mf) {
  constexpr int R = RT_PACKET_RAYS;
  return mf ? reinterpret_cast<const void*>(&k_trace_frame_packet<MODE, false, R, (R == 1 ? KS : 0), true, true>)
            : reinterpret_cast<const void*>(&k_trace_frame_packet<MODE, false, R, (R == 1 ? KS : 0), true, false>);
}
template <int MODE>
const void* bal_kernel_ks(int ks, bool mf) {
  return ks == 1 ? bal_kernel<MODE, 1>(mf) : ks == 2 ? bal_kernel<MODE, 2>(mf) : ks == 4 ? bal_kernel<MODE, 4>(mf)
                                                                                       : bal_kernel<MODE, 0>(mf);
}
}  // namespace

uint32_t trace_wave_slots(const SceneView& sc, const FrameParams& fp, int schedule, int device) {
  const PacketGeometry g = packet_geometry(sc, fp, schedule);
  if (!g.packet) return 0;
  const bool mf = launch_multi_frame(fp);
  const void* k = nullptr;
  switch (fp.shade_mode) {  // the instantiation launch_trace_frame picks (non-STATS, BAL)
    case 0: k = (fp.material.reflectivity == 0.0f && RT_REF_NOREFL) ? bal_kernel_ks<3>(g.ks, mf)
                                                                    : bal_kernel_ks<0>(g.ks, mf);
            break;
    case 1: k = bal_kernel_ks<1>(g.ks, mf); break;
    case 2: k = bal_kernel_ks<2>(g.ks, mf); break;
    default: return 0;
  }
  static std::mutex mu;
  static std::vector<std::pair<std::pair<const void*, int>, uint32_t>> cache;
  std::lock_guard<std::mutex> lk(mu);
  for (const auto& e : cache)
    if (e.first.first == k && e.first.second == device) return e.second;
  const int block = packet_block(RT_PACKET_RAYS == 1 ? g.ks : 0);
  int nb = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, block, 0) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || nb <= 0 || cus <= 0)
    return 0;
  // waves per SIMD: the runtime's figure counts VGPRs and workgroup slots but not the hardware's SGPR budget, which
  // holds these kernels (88 SGPRs) to 7 waves per SIMD where the runtime and the compiler report 8: the wave-time
  // trace finds every one of the 1,024 SIMDs at 7 resident waves, HW wave slots 0..6 (profiles/r05_wave_times_C4.txt),
  // and the register probe puts the limit at 72 SGPRs for 8 waves (tools/occupancy_probe.hip,
  // profiles/r05_occupancy_probe.jsonl). A build capped at 80 SGPRs (72 used) does reach 8 waves but spills 20 SGPRs
  // and is not faster
  const uint32_t per_simd = std::min<uint32_t>((uint32_t)nb * (uint32_t)(block / 64) / 4u, RT_PACKET_HW_WAVES);
  const uint32_t slots = per_simd * 4u * (uint32_t)cus;
  cache.push_back({{k, device}, slots});
  return slots;
}

hipError_t launch_tile_plan(const PlanArgs& a, hipStream_t s) {
  if (a.ntiles > kPlanMaxTiles) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_tile_plan, dim3(1), dim3(kPlanThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_trace_rays(const SceneView& sc, const float* rays, uint32_t n, bool any_hit, bool cull,
                             uint32_t* hits, float* uv, unsigned long long* d_stats, bool stats,
                             hipStream_t s) {
  if (n == 0) return hipSuccess;
  dim3 grid((n + kBlock - 1) / kBlock);
  size_t lds = (size_t)sc.lds_cap * kBlock * sizeof(int);
  const float4* r = (const float4*)rays;
#define RT_LAUNCH_RAYS(A, C, S)                                                                          \
  hipLaunchKernelGGL((k_trace_rays<A, S, C>), grid, dim3(kBlock), lds, s, sc, r, n, (uint4*)hits, (float2*)uv, \
                     d_stats)
  if (any_hit) {
    if (cull) { if (stats) RT_LAUNCH_RAYS(true, true, true); else RT_LAUNCH_RAYS(true, true, false); }
    else { if (stats) RT_LAUNCH_RAYS(true, false, true); else RT_LAUNCH_RAYS(true, false, false); }
  } else {
    if (cull) { if (stats) RT_LAUNCH_RAYS(false, true, true); else RT_LAUNCH_RAYS(false, true, false); }
    else { if (stats) RT_LAUNCH_RAYS(false, false, true); else RT_LAUNCH_RAYS(false, false, false); }
  }
#undef RT_LAUNCH_RAYS
  return hipGetLastError();
}

hipError_t launch_assemble_strips(uint32_t W, uint32_t H, uint32_t nranks, uint32_t strip_rows,
                                  const void* gathered, void* out, hipStream_t s, uint32_t rank_stride_rows,
                                  uint32_t in_bpp) {
  return launch_assemble_frames(W, H, nranks, strip_rows, gathered, &out, 1, 0, s, rank_stride_rows, in_bpp);
}

hipError_t launch_assemble_frames(uint32_t W, uint32_t H, uint32_t nranks, uint32_t strip_rows, const void* gathered,
                                  void* const* outs, uint32_t nframes, size_t frame_bytes, hipStream_t s,
                                  uint32_t rank_stride_rows, uint32_t in_bpp) {
  const uint32_t nstrips = (H + strip_rows - 1) / strip_rows;
  const uint32_t strips_per_rank = (nstrips + nranks - 1) / nranks;
  const uint32_t rows_per_rank = rank_stride_rows ? rank_stride_rows : strips_per_rank * strip_rows;  // rank stride
  if ((in_bpp != 3u && in_bpp != 4u) || nframes == 0 || nframes > (uint32_t)kMaxLaunchFrames) return hipErrorInvalidValue;
  uintptr_t align = ((uintptr_t)gathered | (uintptr_t)frame_bytes) % (in_bpp == 4u ? 16u : 4u);
  for (uint32_t b = 0; b < nframes; ++b) align |= (uintptr_t)outs[b] % 16u;
  if (W % 16 == 0 && H > 0 && W / 16 <= 0xffffffffu / H && ((uintptr_t)gathered | (uintptr_t)frame_bytes) % 16u == 0 &&
      align == 0 && in_bpp == 3u) {  // the strips of rt_comm, 16 pixels per thread: every frame of the batch
    const uint32_t W16 = W / 16;
    AsmFrames f{};
    for (uint32_t b = 0; b < nframes; ++b) f.out[b] = (uint4*)outs[b];
    dim3 grid((W16 * H + 255u) / 256u, 1, nframes);
    hipLaunchKernelGGL(k_assemble48_rgb, grid, dim3(256), 0, s, W16, H, nranks, strip_rows, (const uint4*)gathered, f,
                       rows_per_rank, (uint32_t)(frame_bytes / 16));
    return hipGetLastError();
  }
  if (W % 4 == 0 && align == 0 && in_bpp == 3u) {  // the strips of rt_comm: every frame of the batch in one launch
    const uint32_t W4 = W / 4;
    AsmFrames f{};
    for (uint32_t b = 0; b < nframes; ++b) f.out[b] = (uint4*)outs[b];
    dim3 grid((W4 + 255) / 256, (H + kAsmRows - 1) / kAsmRows, nframes);
    hipLaunchKernelGGL(k_assemble16_rgb, grid, dim3(256), 0, s, W4, H, nranks, strip_rows, (const uint32_t*)gathered,
                       f, rows_per_rank, (uint32_t)(frame_bytes / 4));
    return hipGetLastError();
  }
  for (uint32_t b = 0; b < nframes; ++b) {
    const char* in = (const char*)gathered + b * frame_bytes;
    if (W % 4 == 0 && align == 0) {
      const uint32_t W4 = W / 4;
      dim3 grid((W4 + 255) / 256, (H + kAsmRows - 1) / kAsmRows);
      hipLaunchKernelGGL(k_assemble16, grid, dim3(256), 0, s, W4, H, nranks, strip_rows, (const uint4*)in,
                         (uint4*)outs[b], rows_per_rank);
    } else {
      dim3 grid((W + 255) / 256, H);
      hipLaunchKernelGGL(k_assemble, grid, dim3(256), 0, s, W, H, nranks, strip_rows, (const uint8_t*)in,
                         (uint32_t*)outs[b], rows_per_rank, in_bpp);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace rt
