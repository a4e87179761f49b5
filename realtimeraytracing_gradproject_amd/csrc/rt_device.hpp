// rt_device.hpp — HBM data layout and the per-ray arithmetic of the MI355X trace path.
//
// Everything here is compiled with -ffp-contract=off: the image must be bit-identical to the CPU
// oracle (oracle/rt_oracle.c), which restates the same formulas independently. The only fused
// multiply-adds are the explicit __builtin_fmaf in the slab test, mirrored by the oracle.
//
// Reference semantics (relative to the reference tree):
//   RayGen            shaders/RayGen.hlsl:28-43
//   ray wrappers      shaders/Common.hlsl:44-82
//   ClosestHit & co.  shaders/Hit.hlsl:48-241
//   Miss              shaders/Miss.hlsl:3-10
//   Shadow programs   shaders/ShadowRay.hlsl:10-20
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define RT_HD __host__ __device__ __forceinline__

// Code-shape knobs, A/B-timed in one process with tools/ab.py (results in DESIGN.md §3.2). Each renders the
// identical image; the non-default settings kept in the tree are built and checked against the oracle by
// tests/test_gpu_variants.py (the library variants __graft_entry__.build() compiles). Settings measured slower
// and removed are listed in DESIGN.md §3.2.
#ifndef RT_PACKET_RAYS
#define RT_PACKET_RAYS 1    // rays per lane in a packet (2: 128-ray packets, 8 x 16 pixels per wave)
#endif
// VERDICT r5 #5's LDS candidate, measured slower than the scalar-cache node loads; a variant (ldstop):
#ifndef RT_LDS_TOP
#define RT_LDS_TOP 0        // > 0: the top RT_LDS_TOP BFS nodes of the largest BLAS staged in LDS per packet workgroup
#endif

namespace rt {

// ------------------------------------------------------------------------------------------
// HBM layout
// ------------------------------------------------------------------------------------------

// Binary child-pair node of the Karras LBVH: a build intermediate only (collapsed into Bvh4Node).
// Child refs: >= 0 internal node index, < 0 leaf: ~slot (BLAS: triangle slot in leaf order,
// TLAS: instance index).
struct alignas(64) BinNode {
  float lo0[3], hi0[3];
  float lo1[3], hi1[3];
  int32_t c0, c1;
  uint32_t pad0, pad1;
};
static_assert(sizeof(BinNode) == 64, "BinNode must be 64 B");

// Traversal node: 4-wide, 128 B = one cache line, nodes in BFS order (root 0, then level by
// level: the top of the tree is a contiguous prefix). Child boxes are stored SoA so one node is
// 8 x 16-B loads and the 4 slab tests share per-axis FMAs. Built on the device by collapsing
// the binary LBVH: each wide node opens its largest-area internal descendants until it has 4
// children (fewer only where the subtree runs out of internal nodes).
// child[k]: >= 0 node index, < 0 leaf (~slot / ~instance), kEmptyChild = unused slot.
constexpr int32_t kEmptyChild = INT32_MIN + 1;
struct alignas(128) Bvh4Node {
  float lox[4], hix[4];
  float loy[4], hiy[4];
  float loz[4], hiz[4];
  int32_t child[4];
  uint32_t count;       // valid children
  int32_t first_inner;  // ref of the first internal child (0 when none): the internal children's
                        // refs are consecutive in slot order (BFS allocation); BLAS nodes hold them
                        // in the lowest slots, so there slot k is first_inner + k
  uint32_t inner_mask;  // bit k: child[k] is an internal node (>= 0)
  uint32_t entry_base;  // first_inner << 8 | inner_mask << 4: the packet walk's stack entry for this
                        // node, OR-ed with the pending slots
};
static_assert(sizeof(Bvh4Node) == 128, "Bvh4Node must be 128 B");

// Moller-Trumbore-ready triangle in leaf order, 48 B: v0, e1 = v1 - v0, e2 = v2 - v0, and the
// original PrimitiveIndex().
struct alignas(16) TriRec {
  float v0[3];
  uint32_t prim;
  float e1[3];
  uint32_t pad1;
  float e2[3];
  uint32_t pad2;
};
static_assert(sizeof(TriRec) == 48, "TriRec must be 48 B");

// Per-instance record read by the trace kernel (instance desc + InstanceProperties,
// TopLevelASGenerator.cpp:180-198, Hit.hlsl:19-23).
struct alignas(16) InstanceRec {
  float w2o[12];     // world-to-object 3x4 row-major (inverse of the instance transform)
  float o2w[12];     // object-to-world 3x4 row-major (as given)
  float nrm[9];      // objectToWorldNormal = transpose(inverse(upper3x3)), row-major 3x3
  uint32_t instance_id;
  uint32_t hit_group;
  uint32_t blas;
  const Bvh4Node* nodes;  // the BLAS's own arrays (root = node 0)
  const TriRec* tris;
  uint32_t pool_root;     // the BLAS root's index in the scene pool (see SceneView)
  uint32_t flip;          // instance transform has a negative determinant (front-face sense flipped)
  uint32_t translate;     // upper 3x3 exactly the identity: the object ray is (o + t, d)
  uint32_t pad_;
  const float* vtx;       // 6 floats per vertex: pos.xyz, normal.xyz (stride 24 B)
  const uint32_t* idx;    // triangle list, or nullptr for non-indexed geometry
};

constexpr int kMaxLights = 16;
constexpr int32_t kStackSentinel = INT32_MIN;  // TLAS -> BLAS transition marker
constexpr int kMaxTraversalStack = 256;        // entries per lane (LDS part + HBM overflow)
constexpr int kLdsStackEntries = 32;           // LDS part: 32 KB per 256-lane workgroup
// Packet walks hand a BLAS subtree to per-lane walks when few lanes want it (rt_trace.hip, lane_subtree):
// their stacks live in LDS, kHybridStack entries per lane, so only scenes whose BLAS bound fits take it.
constexpr int kHybridStack = 32;
// Reflection bounces per camera sample in RT_SHADE_REF: the reference pipeline allows 20 nested
// TraceRay levels (D3D12HelloTriangle.cpp:954) = camera ray + 18 reflections + the plane's
// shadow ray. A reflective hit at the limit shades as non-reflective (pinned; DXR would fail).
constexpr int kMaxReflectDepth = 18;

struct LightRec {
  float color[3];
  float position[3];
  float intensity;
};

struct MaterialRec {
  float albedo[3];
  float roughness, metallic, reflectivity;
};

// The material's constants of ClosestHit's surface colour (surface_ref, rt_trace.hip), evaluated once per
// rt_set_shading on the host with the same IEEE float operations the kernel would run per pixel (so the same bits):
// GGX's a^2, Smith's k and 1 - k (Hit.hlsl:104-117), F0 = lerp(0.04, albedo, metallic) (:148-149) and the diffuse
// factor (1 - metallic) albedo / PI (:158-162 as pinned in round 6).
struct SurfaceConsts {
  float a2, k, omk;
  float F0[3];
  float kdA[3];
};
constexpr float kPiF = 3.14159265359f;  // Common.hlsl:1
inline void surface_consts(const MaterialRec& m, SurfaceConsts& c) {
  const float r = m.roughness;
  const float a = r * r;
  c.a2 = a * a;
  const float rp1 = r + 1.0f;
  c.k = (rp1 * rp1) / 8.0f;
  c.omk = 1.0f - c.k;
  const float km = 1.0f - m.metallic;
  for (int i = 0; i < 3; ++i) {
    c.F0[i] = 0.04f + m.metallic * (m.albedo[i] - 0.04f);
    c.kdA[i] = (km * m.albedo[i]) / kPiF;
  }
}

// Frames one launch renders (rt_render_strips_frames: a batch of a tiled-frame loop's frames, one camera each,
// the frame index = blockIdx.z)
constexpr int kMaxLaunchFrames = 4;

// What RayGen reads of one frame's camera buffer (RayGen.hlsl:33-38): viewInverse, projectionInverse (XMMATRIX
// memory order, cb[32..63] of UpdateCameraBuffer) and the origin mul(viewInverse, (0, 0, 0, 1)), evaluated once
// on the host with the device's own arithmetic (a uniform value the kernel would otherwise compute per lane).
struct FrameCam {
  float view_inv[16];
  float proj_inv[16];
  float origin[4];
};

// Everything a frame needs besides the scene buffers; passed by value as a kernel argument.
// (The camera buffer itself stays on the host, rt_ctx::cam_cb: RayGen reads the per-frame FrameCam derived from it,
// and every byte here is kernel-argument data copied per launch.)
struct FrameParams {
  LightRec lights[kMaxLights];
  MaterialRec material;
  SurfaceConsts surf;  // derived from material by rt_set_shading (surface_consts)
  uint32_t nlights;
  uint32_t shade_mode;
  uint32_t spp_side;  // k for k x k stratified samples
  uint32_t width, height;
  uint32_t nrows;
  // the dimensions as floats (frame constants evaluated once on the host)
  float fwidth, fheight;
  uint32_t tile_rows;  // packet schedule, one-sample frames: rows of a wave's 8-wide tile (8 or 4)
  // output format: 4 = RGBA8 (R8G8B8A8_UNORM, D3D12HelloTriangle.cpp:971), 3 = RGB8 (the tiled-frame loop's
  // strips: alpha is the constant 255, restored by the assembly, so a quarter fewer bytes cross xGMI)
  uint32_t out_bpp;
  // frames of the launch (grid z): frame z reads cam[z] and writes its nrows x width pixels frame_bytes * z
  // bytes into the output (the float output, when given, holds frame 0 only)
  uint32_t nframes;
  uint32_t frame_bytes;
  FrameCam cam[kMaxLaunchFrames];
  // Tile balance (packet schedule, rt_set_tile_balance). plan: the launch's wave work list written by k_tile_plan
  // (plan[0] = item count, plan[1 + plan_xaddr(i)] = item i = wave slot << 8 | part << 2 | split code, bit 31 the front class;
  // split code 0: the whole tile, 1: quadrant `part` of 4, 2: cell `part` of 16, 3: pixel `part` of 64), dealt to the waves of a 1-D grid in list order (costliest
  // first), or null: wave slot = the plain grid's wave index. cost: per wave slot, two words written at wave end (or
  // null): [0] the ticks (s_memrealtime) of the tile's last whole wave, bit 31 set by every part of a split since
  // (the whole time is then older than the parts), [1] the costliest part of the tile's last split (ticks << 2 |
  // layout, atomicMax; cleared by the plan that splits the tile). A split tile's current cost is estimated from its
  // parts (k_tile_plan), so a tile that became cheap while split is traced whole again.
  const uint32_t* plan;
  uint32_t* cost;
  uint32_t grid_x;           // workgroups along x of the plain grid
  uint32_t waves_per_frame;  // waves of the plain grid per frame (wave slot = frame * waves_per_frame + ...)
};

// Tile-balance split codes (FrameParams::plan): parts per tile. The costliest quadrant of the costliest C4 tiles
// takes 0.55 of the whole packet's fetches, the costliest 2 x 2 cell 0.35 (tools/split_study.py): the kernel's
// estimate of a whole tile from one part's time, and the plan's estimate of a part from the whole.
RT_HD uint32_t split_parts(uint32_t code) { return code == 0u ? 1u : code == 1u ? 4u : code == 2u ? 16u : 64u; }

// Work-list storage (round 6). The launch deals the list's items to its waves in list order (item p to
// wave p % wl of workgroup p / wl) and the dispatcher deals workgroups round robin over the 8 XCDs, so in list order
// every 64-B line of the list was read by all 8 XCDs' L2s (measured: 1.0 MB of FETCH_SIZE per 1080p launch, C2F and
// C4 alike, with the list equal to the plain order). The items are therefore stored XCD-major: position p lives at
// word plan_xaddr(p), the workgroups of one XCD (linear id = x mod 8) reading a contiguous slice. Only the storage is
// permuted (the plan writes and the launch reads through the same map): the list, its order and the image are not.
RT_HD uint32_t plan_xaddr(uint32_t p, uint32_t wl, uint32_t groups) {
  const uint32_t k = p / wl, j = p - k * wl, per = (groups + 7u) / 8u;
  return ((k & 7u) * per + (k >> 3)) * wl + j;
}
// the workgroups of a launch over a list of `cap` items, and the words its permuted storage spans
RT_HD uint32_t plan_groups(uint32_t cap, uint32_t wl) { return (cap + wl - 1u) / wl; }
RT_HD uint32_t plan_xwords(uint32_t cap, uint32_t wl) { return (plan_groups(cap, wl) + 7u) / 8u * 8u * wl; }

// The trace kernels read one node pool and one triangle pool per scene: [TLAS | BLAS 0 | BLAS 1 ..]
// with child refs rebased to pool indices (BLAS leaves -> ~(global triangle slot)). A uniform base
// (SGPR) plus a 32-bit per-lane byte offset is the global_load saddr form: one VALU add per load
// address instead of 64-bit pointer arithmetic, and per-lane octant offsets pick the near/far
// planes of a node with no min/max.
struct SceneView {
  const Bvh4Node* pool_nodes;
  const TriRec* pool_tris;
  const Bvh4Node* tlas;
  const InstanceRec* inst;
  int stack_cap;       // worst-case entries per lane (exact bound from the trees)
  int packet_cap;      // worst-case entries of the wave-packet stack (TLAS siblings + BLAS levels)
  int lds_cap;         // entries kept in LDS ([entry][lane])
  int* ovf;            // HBM overflow area, [entry - lds_cap][global lane], or null
  uint32_t ovf_lanes;  // lanes of the launch (overflow row pitch)
  float cull_sense;    // culling traces: +1 culls back faces, -1 front faces (DXR ray flags 0x10 / 0x20)
  int hybrid;          // every BLAS's worst-case stack fits kHybridStack: packet walks may hand subtrees to
                       // per-lane walks (lane_subtree)
  int tlas_root;       // the TLAS root's index in the node pool (the TLAS version launches read)
#if RT_LDS_TOP
  int lds_root;  // RT_LDS_TOP experiment: the largest BLAS's root in the pool and how many of its first (BFS)
  int lds_n;     // nodes each packet workgroup copies into LDS (0: none)
#endif
};

// ------------------------------------------------------------------------------------------
// Scalar float helpers (no contraction; identical to oracle/rt_oracle.c)
// ------------------------------------------------------------------------------------------

struct V3 {
  float x, y, z;
};

RT_HD V3 v3(float x, float y, float z) { return V3{x, y, z}; }
RT_HD V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
RT_HD V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
RT_HD V3 mul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
RT_HD V3 muls(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
RT_HD V3 neg(V3 a) { return v3(-a.x, -a.y, -a.z); }
RT_HD float dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
RT_HD V3 cross(V3 a, V3 b) {
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
#ifndef RT_RCP_EXACT
#define RT_RCP_EXACT 2  // 1 / x by rcp + one Newton step (same bits as the division): bit 0 normalize / safe_inv /
                        // shading, bit 1 the triangle test's 1 / det, bit 2 safe_inv alone (the walks' inverse directions)
#endif
// 1 / x, bit-equal to the IEEE quotient `1.0f / x` (what the oracle computes on the CPU) in a third of the
// instructions of the compiler's correctly rounded division (div_scale / rcp / 4 fma / div_fmas / div_fixup):
// v_rcp_f32 (<= 1 ulp) refined by one fused Newton step is bit-equal to 1.0f / x for EVERY float whose biased
// exponent is in [20, 234] (|x| in [2^-107, 2^108); both signs, all 3.6e9 patterns checked on the GPU,
// tools/recip_check.hip). A wave with any lane outside that range (zero, denormal, huge, inf / NaN) takes the
// IEEE division instead, so the result is the IEEE quotient for every input.
RT_HD float rcp_exact(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t b = __builtin_bit_cast(uint32_t, x);
  const bool in = (b << 1) - (20u << 24) < (215u << 24);  // exponent field in [20, 234], sign dropped
  const float r = __builtin_amdgcn_rcpf(x);
  float q = __builtin_fmaf(__builtin_fmaf(-x, r, 1.0f), r, r);
  if (__builtin_amdgcn_ballot_w64(!in)) q = in ? q : 1.0f / x;  // wave-uniform, rare
  return q;
#else
  return 1.0f / x;
#endif
}

// 1 / x of the ray setup and the shading (RT_RCP_EXACT bit 0: rcp_exact; off: the division, same bits)
RT_HD float sh_rcp(float x) {
#if RT_RCP_EXACT & 1
  return rcp_exact(x);
#else
  return 1.0f / x;
#endif
}

// HLSL normalize pinned as v * (1 / sqrt(dot(v, v))) (glm's compute_normalize form).
RT_HD V3 normalize(V3 a) {
  float inv = sh_rcp(sqrtf(dot(a, a)));
  return muls(a, inv);
}
RT_HD float length(V3 a) { return sqrtf(dot(a, a)); }
RT_HD float maxf(float a, float b) { return a > b ? a : b; }
RT_HD float minf(float a, float b) { return a < b ? a : b; }
RT_HD float clamp01(float x) { return minf(maxf(x, 0.0f), 1.0f); }

// 3x4 row-major affine transform of a point / a direction, summed left to right.
RT_HD V3 xform_point(const float* m, V3 p) {
  return v3(((m[0] * p.x + m[1] * p.y) + m[2] * p.z) + m[3],
            ((m[4] * p.x + m[5] * p.y) + m[6] * p.z) + m[7],
            ((m[8] * p.x + m[9] * p.y) + m[10] * p.z) + m[11]);
}
RT_HD V3 xform_dir(const float* m, V3 d) {
  return v3((m[0] * d.x + m[1] * d.y) + m[2] * d.z, (m[4] * d.x + m[5] * d.y) + m[6] * d.z,
            (m[8] * d.x + m[9] * d.y) + m[10] * d.z);
}
// World -> object ray of an instance. A pure translation moves the origin only: the general
// product costs 33 operations (and turns a -0 direction component into +0; safe_inv maps both
// zeros to +1e20, so the inverse direction is the world ray's).
RT_HD V3 inst_point(const float* m, uint32_t translate, V3 p) {
  return translate ? v3(p.x + m[3], p.y + m[7], p.z + m[11]) : xform_point(m, p);
}
RT_HD V3 inst_dir(const float* m, uint32_t translate, V3 d) { return translate ? d : xform_dir(m, d); }
RT_HD V3 mat3_mul(const float* m, V3 d) {
  return v3((m[0] * d.x + m[1] * d.y) + m[2] * d.z, (m[3] * d.x + m[4] * d.y) + m[5] * d.z,
            (m[6] * d.x + m[7] * d.y) + m[8] * d.z);
}

// HLSL mul(M, v) with M read column-major from XMMATRIX memory: r_i = sum_j mem[4j+i] v_j.
RT_HD void hlsl_mul4(const float* mem, const float v[4], float r[4]) {
  for (int i = 0; i < 4; ++i)
    r[i] = ((mem[i] * v[0] + mem[4 + i] * v[1]) + mem[8 + i] * v[2]) + mem[12 + i] * v[3];
}

// 1/d with zero components replaced by +-1e20 so slab products never form inf*0.
RT_HD float safe_inv(float d) {
  const bool big = fabsf(d) > 1e-20f;
#if RT_RCP_EXACT & 4
  const float q = rcp_exact(big ? d : 1.0f);  // the replaced components never send the wave to the slow path
#else
  const float q = sh_rcp(big ? d : 1.0f);
#endif
  return big ? q : (d < 0.0f ? -1e20f : 1e20f);
}

// Deterministic log2 / exp2 / pow for x in [0, inf): pure +,-,*,/ and bit operations so the GPU
// and the oracle agree to the bit. |rel err| ~ 2e-7.
RT_HD float det_log2(float x) {
  uint32_t b = __builtin_bit_cast(uint32_t, x);
  int e = (int)((b >> 23) & 0xffu) - 127;
  float m = __builtin_bit_cast(float, (b & 0x7fffffu) | 0x3f800000u);
  if (m > 1.41421356f) {
    m = m * 0.5f;
    e = e + 1;
  }
  float f = m - 1.0f;
  float s = f * rcp_exact(2.0f + f);  // 2 + f in [1.7, 2.5]: rcp_exact's fast path, the IEEE 1 / (2 + f)
  float s2 = s * s;
  float p = 1.0f / 11.0f;
  p = p * s2 + 1.0f / 9.0f;
  p = p * s2 + 1.0f / 7.0f;
  p = p * s2 + 1.0f / 5.0f;
  p = p * s2 + 1.0f / 3.0f;
  p = p * s2 + 1.0f;
  float ln = (2.0f * s) * p;
  return (float)e + ln * 1.44269504f;
}
RT_HD float det_exp2(float y) {
  if (y < -126.0f) return 0.0f;
  if (y > 127.0f) y = 127.0f;
  float fi = floorf(y + 0.5f);
  float f = y - fi;  // [-0.5, 0.5]
  float a = f * 0.693147181f;
  float p = 1.0f / 40320.0f;
  p = p * a + 1.0f / 5040.0f;
  p = p * a + 1.0f / 720.0f;
  p = p * a + 1.0f / 120.0f;
  p = p * a + 1.0f / 24.0f;
  p = p * a + 1.0f / 6.0f;
  p = p * a + 0.5f;
  p = p * a + 1.0f;
  p = p * a + 1.0f;
  int i = (int)fi;
  float scale = __builtin_bit_cast(float, (uint32_t)(i + 127) << 23);
  return p * scale;
}
RT_HD float det_pow(float x, float y) {
  if (!(x > 1e-30f)) return 0.0f;
  return det_exp2(y * det_log2(x));
}

// float -> UNORM8 (D3D conversion: saturate, x255, round to nearest; NaN -> 0).
RT_HD uint32_t unorm8(float c) {
  if (!(c > 0.0f)) return 0u;
  if (c >= 1.0f) return 255u;
  return (uint32_t)(c * 255.0f + 0.5f);
}

// Slab tests of the 4 children of a Bvh4Node against the ray segment [tmin, tbest], given each
// axis's near and far planes (the ray's octant picks them: near = lo where invd >= 0, else hi).
// tn[k] = entry distance of child k, or +inf if it is missed or empty. Conservative (tfar
// widened by 1 + 4e-7) so BVH culling never rejects a triangle Moller-Trumbore accepts.
// Bitwise equal to the min/max form of oracle oslab4: for invd > 0 the exact products lo*invd <=
// hi*invd and the fma rounding is monotone, so fma(lo,..) <= fma(hi,..) (reversed for invd < 0;
// safe_inv never returns 0), i.e. min/max of the two plane distances is the near/far plane.
RT_HD void slab4_octant(const float* nx, const float* fx, const float* ny, const float* fy,
                        const float* nz, const float* fz, const int32_t* child, V3 invd, V3 noinv,
                        float tmin, float tbest, float tn[4]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float tnx = __builtin_fmaf(nx[k], invd.x, noinv.x), tfx = __builtin_fmaf(fx[k], invd.x, noinv.x);
    const float tny = __builtin_fmaf(ny[k], invd.y, noinv.y), tfy = __builtin_fmaf(fy[k], invd.y, noinv.y);
    const float tnz = __builtin_fmaf(nz[k], invd.z, noinv.z), tfz = __builtin_fmaf(fz[k], invd.z, noinv.z);
    const float n = fmaxf(fmaxf(tnx, tny), fmaxf(tnz, tmin));
    const float f = fminf(fminf(tfx, tfy), fminf(tfz, tbest));
    (void)child;  // unused slots carry +inf boxes, rejected here like any missed child
    tn[k] = n <= f * 1.0000004f ? n : __builtin_inff();
  }
}

// Orders 4 (distance, ref) pairs ascending with the 5-comparator network (0,1)(2,3)(0,2)(1,3)(1,2);
// a pair moves only when strictly nearer, so equal distances keep a fixed, shared order.
RT_HD void cswap(float& ta, int32_t& ra, float& tb, int32_t& rb) {
  const bool s = tb < ta;
  const float t = s ? tb : ta;
  const int32_t r = s ? rb : ra;
  tb = s ? ta : tb;
  rb = s ? ra : rb;
  ta = t;
  ra = r;
}
RT_HD void sort4(float t[4], int32_t r[4]) {
  cswap(t[0], r[0], t[1], r[1]);
  cswap(t[2], r[2], t[3], r[3]);
  cswap(t[0], r[0], t[2], r[2]);
  cswap(t[1], r[1], t[3], r[3]);
  cswap(t[1], r[1], t[2], r[2]);
}

// dot / cross for the triangle test: cross products fused (fma(a.y, b.z, -(a.z * b.y)) ...), dot products
// unfused, mirrored bit for bit by the oracle's omt_cross / omt_dot (as the slab test's fmas are by oslab4).
// profiles/r03_ab_mt_fma.txt: fused cross 1-2% faster frames with the seam-probe leak count nearly unchanged
// (1727 -> 1832 of 66,304 edge rays, pinned by tests/test_oracle.py); fusing the dots as well gained 2-4% but
// raised it to 2514, so they stay unfused (a deliberate deviation from DXR's watertight test).
RT_HD float mt_dot(V3 a, V3 b) { return dot(a, b); }
RT_HD V3 mt_cross(V3 a, V3 b) {
  return v3(__builtin_fmaf(a.y, b.z, -(a.z * b.y)), __builtin_fmaf(a.z, b.x, -(a.x * b.z)),
            __builtin_fmaf(a.x, b.y, -(a.y * b.x)));
}

// The culling term of the triangle test: det * face < 0 rejects. With face == 0 (no culling: primary and shadow
// rays) det * 0 is +-0 or NaN, never < 0, so the term is always false; written so the compiler folds it away when
// face is the constant 0 after inlining (it does not fold x * 0 < 0 itself) instead of a multiply and a compare.
RT_HD bool culled(float det, float face) { return face != 0.0f && det * face < 0.0f; }

// 1 / det of the triangle test (RT_RCP_EXACT bit 1: rcp_exact; off: the division, same bits)
RT_HD float mt_rcp(float det) {
#if RT_RCP_EXACT & 2
  return rcp_exact(det);
#else
  return 1.0f / det;
#endif
}

// Moller-Trumbore. Accepts u >= 0, v >= 0, u + v <= 1, det != 0; returns t (not yet range checked).
// face: 0 accepts both sides; +1 / -1 accepts only det * face > 0, i.e. front faces under DXR's
// RAY_FLAG_CULL_BACK_FACING_TRIANGLES (front = clockwise seen from the ray origin = det > 0 with
// det = e1 . (d x e2), the sense flipped by a negative instance-transform determinant: face = -1).
RT_HD bool moller_trumbore(V3 o, V3 d, V3 v0, V3 e1, V3 e2, float face, float& t, float& u, float& v) {
  V3 p = mt_cross(d, e2);
  float det = mt_dot(e1, p);
  if (det == 0.0f || culled(det, face)) return false;
  float inv = mt_rcp(det);
  V3 s = sub(o, v0);
  u = mt_dot(s, p) * inv;
  if (!(u >= 0.0f && u <= 1.0f)) return false;
  V3 q = mt_cross(s, e1);
  v = mt_dot(d, q) * inv;
  if (!(v >= 0.0f && u + v <= 1.0f)) return false;
  t = mt_dot(e2, q) * inv;
  return true;
}

// Moller-Trumbore without early exits: every lane runs the same instructions (the wave-packet
// path, where a divergent early exit costs exec-mask SALU work on the busiest pipe). Accepts
// exactly what moller_trumbore accepts, with the same u, v, t.
RT_HD bool moller_trumbore_flat(V3 o, V3 d, V3 v0, V3 e1, V3 e2, float face, float& t, float& u, float& v) {
  const V3 p = mt_cross(d, e2);
  const float det = mt_dot(e1, p);
  const float inv = mt_rcp(det);
  const V3 s = sub(o, v0);
  u = mt_dot(s, p) * inv;
  const V3 q = mt_cross(s, e1);
  v = mt_dot(d, q) * inv;
  t = mt_dot(e2, q) * inv;
  // Bitwise & (no exec-mask region), with two terms fewer than the early-exit form. u <= 1 is implied: v >= 0
  // (not NaN) makes u + v >= u exactly, and rounding is monotone, so fl(u + v) <= 1 gives u <= 1 (a NaN u fails
  // u + v <= 1). min(u, v) >= 0 is u >= 0 and v >= 0 for non-NaN u, v (-0 included); a NaN one (the min returns
  // the other) fails u + v <= 1 anyway (tests/test_acceptance.py).
  return (det != 0.0f) & !culled(det, face) & (__builtin_fminf(u, v) >= 0.0f) & (u + v <= 1.0f);
}

// HLSL reflect(i, n) = i - 2 * n * dot(i, n), evaluated as i - (2 n) * dot(i, n).
RT_HD V3 reflect_dir(V3 i, V3 n) {
  const float t = dot(i, n);
  return v3(i.x - (2.0f * n.x) * t, i.y - (2.0f * n.y) * t, i.z - (2.0f * n.z) * t);
}

}  // namespace rt
