// rt_internal.hpp — launchers shared between the C-ABI (rt_api.cpp) and the HIP translation units.
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/rt_api.h"
#include "rt_device.hpp"

namespace rt {

// --- context accessors for the other host translation units (rt_comm.cpp) ---------------------
int ctx_device(rt_ctx* c);
// a fresh row-list generation (the tile balance keys a launch shape on the row list's pointer AND generation: a
// buffer re-used for another list is another shape)
uint64_t ctx_next_rows_gen(rt_ctx* c);
void* ctx_stream(rt_ctx* c);
// rt_dispatch_rays' argument / scene checks and its launch with a device row list (rt_render_strips keeps its
// rank's rows on the device and skips the host list's upload ring)
rt_status check_dispatch(rt_ctx* c, uint32_t W, uint32_t H, const void* rgba8, bool cameras_given = false);
// nframes (1 .. kMaxLaunchFrames) frames in one launch, frame z with camera buffer cams[64 z ..] (null: the
// context's camera) into rgba8 + z * frame_stride bytes (0: nrows * W * out_bpp); out_bpp 4 = RGBA8, 3 = RGB8
// (the strips of rt_comm)
rt_status dispatch_frame(rt_ctx* c, uint32_t W, uint32_t H, const uint32_t* d_rows, uint32_t nrows, void* rgba8,
                         float* rgba32f, hipStream_t s, uint32_t out_bpp, uint32_t nframes, const float* cams,
                         uint64_t frame_stride, uint64_t rows_gen);
// A stream that launched work on the context is going away (rt_forget_stream): the TLAS version it read gets
// that stream's completion event now, so a later rt_tlas_build never records on the destroyed handle.
hipError_t ctx_forget_stream(rt_ctx* c, hipStream_t s);

// --- LBVH build (rt_lbvh.hip) ---------------------------------------------------------------

// Builds an LBVH over n primitive boxes (d_primbox: n x {lo.xyz, hi.xyz}) and collapses it into
// 4-wide BFS-ordered nodes. d_nodes needs room for max(n-1, 1) nodes (an upper bound); the count
// used, the number of levels and the worst-case traversal stack of the tree are returned, with
// the root box, in host memory. d_sorted
// receives the leaf-order -> primitive permutation. Leaf refs are ~leaf_slot (BLAS, primitives
// reordered afterwards) or ~primitive (TLAS). With d_tri_in the BLAS triangles are gathered into
// leaf order (d_tri_out) as part of the build. Synchronous.
// Device scratch of lbvh_build kept between builds (a per-frame TLAS update must not hipMalloc / hipFree:
// both synchronise the device). Grown on demand; release() frees it.
struct BuildArena {
  void* p = nullptr;
  size_t cap = 0;
  hipEvent_t e0 = nullptr, e1 = nullptr;  // build timing
  void* host = nullptr;                    // pinned readback of the build's bounds + node count / depth / stack
  void release() {
    if (p) (void)hipFree(p);
    if (host) (void)hipHostFree(host);
    host = nullptr;
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    p = nullptr;
    cap = 0;
    e0 = e1 = nullptr;
  }
};

hipError_t lbvh_build(const float* d_primbox, uint32_t n, Bvh4Node* d_nodes, uint32_t* d_sorted,
                      bool leaf_ref_is_prim, uint32_t* node_count, uint32_t* depth, uint32_t* max_stack,
                      float bounds[6], float* build_ms, hipStream_t stream, const TriRec* d_tri_in = nullptr,
                      TriRec* d_tri_out = nullptr, BuildArena* arena = nullptr);

// Triangle setup: prim boxes + unsorted MT records from a {pos, normal} vertex array.
hipError_t blas_prepare(const float* d_vtx, const uint32_t* d_idx, uint32_t ntri, TriRec* d_tris,
                        float* d_primbox, hipStream_t stream);
// Gathers triangles into leaf order.
hipError_t blas_reorder(const TriRec* d_in, const uint32_t* d_sorted, uint32_t n, TriRec* d_out,
                        hipStream_t stream);
// Copies n nodes into the scene pool at dst, rebasing internal refs by node_base and leaf refs
// (~slot) by tri_base (TLAS: node_base = 0, tri_base = -1 keeps ~instance refs).
hipError_t pool_rebase(const Bvh4Node* src, uint32_t n, uint32_t node_base, int64_t tri_base, Bvh4Node* dst,
                       hipStream_t stream);
// World boxes of instances: the 8 corners of each BLAS root box through the instance transform.
hipError_t tlas_prepare(const InstanceRec* d_inst, const float* d_blas_bounds, uint32_t n,
                        float* d_primbox, hipStream_t stream);

// --- Trace (rt_trace.hip) -------------------------------------------------------------------

// plan_items: with fp.plan set, the waves of the launch's 1-D grid (the work list's budget: tiles + parts)
hipError_t launch_trace_frame(const SceneView& scene, const FrameParams& fp, const uint32_t* d_rows,
                              void* rgba8, float* rgba32f, unsigned long long* d_stats, bool stats,
                              int schedule, uint32_t plan_items, hipStream_t stream);

// The packet kernel's plain grid for a launch (schedule, tile layout), or packet = false (the per-lane kernel).
struct PacketGeometry {
  bool packet = false;
  int ks = 1;                          // samples of a pixel in consecutive lanes (1, 2, 4), 0: the sample loop
  uint32_t grid_x = 0, grid_y = 0;     // workgroups of one frame
  uint32_t wx = 1, wy = 1, wl = 1;     // waves of a workgroup along x, y; total
  uint32_t waves_per_frame = 0;
  uint32_t kmax_code = 0;              // largest tile-balance split code the tile allows (0: none, 1: 4, 2: 16, 3: 64)
  bool plannable = false;              // a work list may drive the launch
};
PacketGeometry packet_geometry(const SceneView& sc, const FrameParams& fp, int schedule);
// The GPU's wave slots for the packet kernel a tile-balance launch of this shape runs (the recording / list
// instantiation): hipOccupancyMaxActiveBlocksPerMultiprocessor of that kernel x waves per workgroup x the device's
// CUs, cached per (kernel, device); 0 if the runtime cannot tell.
uint32_t trace_wave_slots(const SceneView& sc, const FrameParams& fp, int schedule, int device);

// Tile balance (k_tile_plan): the summary the plan kernel leaves in host-mapped memory for the next dispatches.
struct PlanStats {
  uint32_t nitems, nsplit, want_extra, max_cost, mean_cost, threshold, plans;
  uint32_t pays;  // the last plan found the costliest tile above the load bound (its list is not the plain order)
  // PlanArgs::check: tiles whose items were not exactly one layout's parts, summed over the plans; the first one
  uint32_t bad, first_bad_tile, first_bad_word;
  uint32_t phase_ticks[3];  // the last plan's phases: snapshot + load bound, budget, placement (10-ns ticks)
  uint32_t coherent;        // the last plan found every measured split useless (it split nothing)
  // items the plans could not place inside the list's budget (summed), and the plans that therefore fell back to the
  // plain grid's list (every tile whole, in order): the budget loop should make both 0 (loud, not a
  // silently dropped part)
  uint32_t refused, refused_plans;
  uint32_t slots;           // the wave slots the last plan's load bound divided by (PlanArgs::slots)
};
struct PlanArgs {
  uint32_t* cost;         // per wave slot of the plain grid, 2 words: the last whole wave's time (ticks), the
                          // costliest part of the last split (time << 2 | layout; cleared here when splitting)
  uint32_t* plan;         // out: [0] item count, [1 ..] items (ntiles + extra_cap words), then the cover check's
                          // scratch (3 ntiles words): 1 + 4 ntiles + extra_cap words in all
  PlanStats* stats;       // host-mapped, or null
  uint32_t ntiles;        // wave slots of the plain grid, every frame of the launch
  uint32_t extra_cap;     // items beyond ntiles the launch's grid has waves for
  uint32_t slots;         // wave slots of the GPU for the list's trace kernel: its occupancy (waves per CU, from the
                          // runtime for the instantiation launched) x CUs (trace_wave_slots)
  uint32_t kmax_code;
  uint32_t force;         // 0 adaptive; 1 / 2 / 3 forced layouts (tests)
  uint32_t split;         // adaptive: split tiles (0: order only)
  uint32_t front;         // adaptive: items estimated above front / 16 x the load bound go first (0: tile order)
  uint32_t check;         // diagnostics: verify the list covers every tile once (PlanStats::bad)
  uint32_t min_gain;      // adaptive: ticks the costliest tile must outlast the load bound by (the plan's own time)
  uint32_t prio;          // adaptive: mark the front class's items (bit 31): their waves raise their issue priority
  uint32_t waves_per_frame, grid_x, wx, wy, wl;
};
// one workgroup holding the costs in registers: launches of at most kPlanMaxTiles wave slots
constexpr uint32_t kPlanMaxTiles = 32u * 1024u;
// work-list items: wave slot << 8 | part << 2 | split code, bit 31 the front class (PlanArgs::prio)
constexpr uint32_t kPlanSlotMask = 0x7fffffu;
hipError_t launch_tile_plan(const PlanArgs& a, hipStream_t stream);

hipError_t launch_trace_rays(const SceneView& scene, const float* rays, uint32_t n, bool any_hit, bool cull,
                             uint32_t* hits, float* uv, unsigned long long* d_stats, bool stats,
                             hipStream_t stream);

// rank_stride_rows: rows from one rank's block of `gathered` to the next (0: rows_per_rank, one frame per block;
// a batched gather holds several frames per rank block and passes their total)
// in_bpp: bytes per pixel of the gathered strips (4 RGBA8, 3 RGB8: the alpha byte restored as 255); out is RGBA8
hipError_t launch_assemble_strips(uint32_t W, uint32_t H, uint32_t nranks, uint32_t strip_rows,
                                  const void* gathered, void* out, hipStream_t stream, uint32_t rank_stride_rows = 0,
                                  uint32_t in_bpp = 4);
// The frames of a batched gather: frame b's strips start b x frame_bytes into every rank's block of `gathered`
// (rank stride rank_stride_rows rows); RGB8 strips of a 4-aligned width go in ONE launch (grid z = frame).
hipError_t launch_assemble_frames(uint32_t W, uint32_t H, uint32_t nranks, uint32_t strip_rows, const void* gathered,
                                  void* const* outs, uint32_t nframes, size_t frame_bytes, hipStream_t stream,
                                  uint32_t rank_stride_rows, uint32_t in_bpp);

// --- Raster fallback (rt_raster.hip) -------------------------------------------------------

constexpr uint32_t kRasterMaxDraws = 8;
constexpr unsigned long long kRasterClear = ~0ull;  // (depth, primitive) of an untouched pixel

struct RasterDraws {  // draw list in submission order; primitive id = first[d] + local triangle
  uint32_t n = 0, total = 0;
  uint32_t first[kRasterMaxDraws] = {};
  uint32_t nvtx[kRasterMaxDraws] = {};
  const float* vtx[kRasterMaxDraws] = {};    // {pos, normal} x nvtx (the reference Vertex)
  const uint32_t* idx[kRasterMaxDraws] = {};  // nullptr: non-indexed draw
};

struct RasterView {
  float o2w[16];   // instance 0 objectToWorld, XMMATRIX memory (row-vector convention)
  float view[16];  // camera buffer view (cb[0..15])
  float proj[16];  // camera buffer projection (cb[16..31])
  uint32_t width, height;
};

struct RasterSlot {  // one screen-space triangle after clipping (48 B)
  int32_t x[3], y[3];  // 16.8 fixed point
  float z[3];
  uint32_t prim;
  uint16_t tx0, ty0, tw, th;  // 8x8-pixel tile box
};

struct RasterScratch {
  float4* clip = nullptr;       // 3 clip-space vertices per primitive
  RasterSlot* slots = nullptr;  // 7 per primitive
  uint32_t* tiles = nullptr;    // tile-box size per slot
  uint32_t* tcount = nullptr;   // per screen tile: binned triangles (then the append cursor)
  uint32_t* toffs = nullptr;    // exclusive scan of tcount, + total (screen tiles + 1)
  uint32_t* bins = nullptr;     // slot ids grouped by screen tile
  uint32_t* bsum = nullptr;     // scan block sums (screen tiles / 4096 + 1)
  RasterDraws* draws = nullptr; // device copy of the draw list
};

// Phase 1: vertex stage, clipping, setup and bin counting; toffs[ntiles] = number of bin entries.
// Phase 2: bin fill + per-tile raster and shading. `bins` holds bin_cap entries: a draw with more
// entries leaves the bins unfilled and every tile walks the whole slot list (same image, slower).
hipError_t launch_raster_bin(const RasterDraws& dr, const RasterView& rv, const RasterScratch& s,
                             hipStream_t stream);
hipError_t launch_raster_draw(const RasterDraws& dr, const RasterView& rv, const RasterScratch& s, uint32_t bin_cap,
                              void* rgba8, float* depth, hipStream_t stream);

}  // namespace rt
