// rt_api.cpp — C-ABI implementation: contexts, BLAS/TLAS lifetimes, frame state and launches.
// No exception crosses the boundary; every failure returns an rt_status and sets rt_last_error.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt_api.h"
#include "rt_internal.hpp"

namespace {

struct DeviceBlas {
  rt::Bvh4Node* nodes = nullptr;
  rt::TriRec* tris = nullptr;
  float* vtx = nullptr;
  uint32_t* idx = nullptr;
  uint32_t ntri = 0, nnodes = 0, depth = 0, nvtx = 0, max_stack = 0;
  float bounds[6] = {0, 0, 0, 0, 0, 0};
  double build_ms = 0.0;
  void release() {
    if (nodes) (void)hipFree(nodes);
    if (tris) (void)hipFree(tris);
    if (vtx) (void)hipFree(vtx);
    if (idx) (void)hipFree(idx);
    nodes = nullptr;
    tris = nullptr;
    vtx = nullptr;
    idx = nullptr;
  }
};

// Device scratch that launches on different streams may need at the same time (the HBM
// overflow stack of the per-lane traversal, the row list of a strip dispatch). The calls are
// stream-ordered and asynchronous (rt_api.h), so one buffer per context would be written by two
// frames in flight at once. Each buffer is a slot of a small ring; a slot remembers, per stream,
// an event recorded after that stream's last launch that used it. A launch on stream s:
//   - takes a slot no other stream is still using (its events have completed), or that only s
//     used (stream order protects it), else a new slot (up to kMaxSlots);
//   - with every slot busy, reuses the least recently used one after making s WAIT (on the
//     device, hipStreamWaitEvent) for the other streams' last uses of it.
// The host never waits except to grow a slot (rare: its old buffer is freed).
struct StreamUse {
  hipStream_t stream;
  hipEvent_t ev;
};

struct ScratchSlot {
  void* buf = nullptr;
  size_t cap = 0;               // bytes
  uint64_t tick = 0;            // last acquisition (LRU)
  std::vector<StreamUse> uses;  // one entry per stream that used the slot
  // row-list slots: the list held (content key), its pinned upload staging and the upload's event
  std::vector<uint32_t> key;
  uint32_t* staging = nullptr;
  size_t staging_cap = 0;
  hipEvent_t upload_ev = nullptr;
  hipStream_t upload_stream = nullptr;
  bool uploaded = false;  // an upload may still be pending (upload_ev not yet seen complete)
  uint64_t gen = 0;       // row-list slots: the context's generation of the list held (new at every upload)
};

struct ScratchRing {
  static constexpr size_t kMaxSlots = 8;
  std::vector<ScratchSlot> slots;
  uint64_t clock = 0;
};

hipEvent_t new_sync_event() {
  hipEvent_t e = nullptr;
  // no timestamp, no system-scope release: the consumers are device-side waits and host queries of completion
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess) return nullptr;
  return e;
}

// true when no stream other than s may still be using the slot
bool slot_free_for(const ScratchSlot& sl, hipStream_t s) {
  for (const StreamUse& u : sl.uses)
    if (u.stream != s && hipEventQuery(u.ev) != hipSuccess) return false;
  return true;
}

// stream s waits (on the device) for every other stream's last use of the slot
hipError_t slot_order_after_others(const ScratchSlot& sl, hipStream_t s) {
  for (const StreamUse& u : sl.uses)
    if (u.stream != s) {
      hipError_t e = hipStreamWaitEvent(s, u.ev, 0);
      if (e != hipSuccess) return e;
    }
  return hipSuccess;
}

// the host waits for every use of the slot (before its buffer is freed)
hipError_t slot_drain(const ScratchSlot& sl) {
  for (const StreamUse& u : sl.uses) {
    hipError_t e = hipEventSynchronize(u.ev);
    if (e != hipSuccess) return e;
  }
  if (sl.upload_ev && sl.uploaded) return hipEventSynchronize(sl.upload_ev);
  return hipSuccess;
}

// records that a launch just enqueued on s used the slot
hipError_t slot_mark_use(ScratchSlot& sl, hipStream_t s) {
  for (StreamUse& u : sl.uses)
    if (u.stream == s) return hipEventRecord(u.ev, s);
  // forget streams whose last use completed long ago (streams come and go: torch, callers)
  if (sl.uses.size() >= 8) {
    std::vector<StreamUse> keep;
    for (const StreamUse& u : sl.uses) {
      if (hipEventQuery(u.ev) == hipSuccess) (void)hipEventDestroy(u.ev);
      else keep.push_back(u);
    }
    sl.uses.swap(keep);
  }
  hipEvent_t ev = new_sync_event();
  if (!ev) return hipErrorOutOfMemory;
  sl.uses.push_back({s, ev});
  return hipEventRecord(ev, s);
}

void slot_release(ScratchSlot& sl) {
  if (sl.buf) (void)hipFree(sl.buf);
  if (sl.staging) (void)hipHostFree(sl.staging);
  for (const StreamUse& u : sl.uses) (void)hipEventDestroy(u.ev);
  if (sl.upload_ev) (void)hipEventDestroy(sl.upload_ev);
  sl = ScratchSlot();
}

// One TLAS version: device instance records, the raw TLAS (export), its slot in the scene pool, pinned
// upload staging, and the uses of the version by launches (a ScratchSlot's per-stream events).
struct TlasVersion {
  rt::Bvh4Node* nodes = nullptr;  // as built (child refs local to the TLAS), for rt_tlas_export
  rt::InstanceRec* inst = nullptr;
  uint32_t* sorted = nullptr;
  uint32_t cap = 0;               // instances the arrays hold
  uint32_t ninst = 0, nodes_n = 0, depth = 0, max_stack = 0;
  float bounds[6] = {0, 0, 0, 0, 0, 0};
  double ms = 0.0;
  uint32_t pool_base = 0;         // this version's TLAS root in the scene pool
  bool valid = false;             // built against the current pool layout
  std::vector<rt_instance> host;  // the instances as given
  rt::InstanceRec* staging = nullptr;  // pinned upload staging (records, then BLAS boxes)
  size_t staging_bytes = 0;
  ScratchSlot use;                // launches that read this version: per-stream events, recorded when it stops being current
  std::vector<hipStream_t> readers;  // streams that launched with it since it became current (no event per launch)
  hipEvent_t ready = nullptr;     // recorded on the context stream when the version's pool slot is written
  bool ready_pending = false;     // launches on other streams still wait for `ready`
  void release() {
    if (nodes) (void)hipFree(nodes);
    if (inst) (void)hipFree(inst);
    if (sorted) (void)hipFree(sorted);
    if (staging) (void)hipHostFree(staging);
    if (ready) (void)hipEventDestroy(ready);
    slot_release(use);
    *this = TlasVersion();
  }
};

// A launch on s that read TLAS version v is noted host-side only (note_reader); when v stops being current,
// one event per reader stream is recorded (note_swap_out): it covers every earlier launch on that stream, so a
// later build into v orders after all of them without an event record per launch.
// The readers list is cleared on every path: a failed record (a stream the caller destroyed without
// rt_forget_stream) would otherwise fail every later update. After a failure the launches of the failed readers
// are not covered by an event, so the device is drained instead (their buffers may be rewritten next).
hipError_t note_swap_out(TlasVersion& v) {
  hipError_t first = hipSuccess;
  for (hipStream_t r : v.readers) {
    const hipError_t e = slot_mark_use(v.use, r);
    if (e != hipSuccess && first == hipSuccess) first = e;
  }
  v.readers.clear();
  if (first != hipSuccess) (void)hipDeviceSynchronize();
  return first;
}

hipError_t note_reader(TlasVersion& v, hipStream_t s) {
  for (hipStream_t r : v.readers)
    if (r == s) return hipSuccess;
  // many streams (a caller creating streams as it goes): record the uses so far now, keep the list short
  if (v.readers.size() >= 16) {
    hipError_t e = note_swap_out(v);
    if (e != hipSuccess) return e;
  }
  v.readers.push_back(s);
  return hipSuccess;
}

// Tile balance (rt_set_tile_balance) of one launch shape (frame size, row list, frames per launch, tile layout):
// the per-tile wave times the packet kernel leaves (FrameParams::cost), the plan kernel's summary in host-mapped
// memory, the work list's budget of extra waves for split tiles, and the shape's work lists. A list is a valid
// cover of the shape's tiles whatever costs it was planned from, so launches reuse the current one, the plan kernel
// runs again only every few launches (balance_wants_plan), and it runs OFF the launches' streams: on the context's
// own stream (a further stream would change which of the caller's streams share a hardware queue), and a launch
// switches to the new list once a host query finds its plan complete (no launch ever waits for a plan). Two lists: the current one, and the other — the one before it, which launches on
// other streams may still be reading; the next plan overwrites it, ordered after them.
struct BalanceMap {
  uint32_t W = 0, nrows = 0, nframes = 0, tile_rows = 0, spp = 0, ntiles = 0;
  const uint32_t* rows = nullptr;
  uint64_t rows_gen = 0;             // the row list's generation (a ring slot re-used for another list is a new shape)
  uint32_t* cost = nullptr;          // device: 2 words per tile (whole wave time, costliest part; PlanArgs)
  uint32_t cost_cap = 0;             // tiles the cost buffer holds (a recycled map keeps it)
  std::vector<hipStream_t> streams;  // every stream that launched reading or writing the map's buffers
  rt::PlanStats* stats = nullptr;    // host-mapped, written by k_tile_plan
  rt::PlanStats* stats_dev = nullptr;
  uint32_t extra_cap = 0;
  uint64_t launches = 0, tick = 0;   // launches: those with the balance active
  hipStream_t last_stream = nullptr; // the stream of the shape's previous launch (cleared by rt_forget_stream)
  uint32_t active_run = 0;           // launches in a row with the balance active
  uint32_t idle_queries = 0;         // launches in flight since the last stream query
  ScratchSlot list[2];               // work lists; uses recorded when a list stops being current
  int cur = -1;                      // the current list (its plan complete), or none
  uint32_t cur_items = 0;            // its launch's grid budget (tiles + extra waves)
  int pending = -1;                  // the list a plan kernel is writing, or none
  uint32_t pending_items = 0;
  uint64_t planned_at = 0;           // launches of the shape when the last plan started
  hipEvent_t pend_ev = nullptr;      // recorded on the plan stream after the pending plan
  hipEvent_t src_ev = nullptr;       // recorded on the launch's stream: the plan starts after its earlier work
  std::vector<hipStream_t> readers;  // streams that launched with the current list since it became current
  ScratchSlot forgotten;             // events on streams dropped by rt_forget_stream (their launches may still run)
  bool recycled = false, recycled_planned = false;  // reused for this shape; a plan has started on it since
  uint32_t nopay_run = 0;            // consecutive completed plans whose list did not pay (re-check back-off)
  void release() {
    if (cost) (void)hipFree(cost);
    if (stats) (void)hipHostFree(stats);
    slot_release(list[0]);
    slot_release(list[1]);
    slot_release(forgotten);
    if (pend_ev) (void)hipEventDestroy(pend_ev);
    if (src_ev) (void)hipEventDestroy(src_ev);
    *this = BalanceMap();
  }
};

}  // namespace

struct rt_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  std::vector<DeviceBlas> blas;
  // TLAS: two versions (double buffering, as the reference's per-frame update of the instance buffer
  // behind its fences, D3D12HelloTriangle.cpp:421-433 / TopLevelASGenerator.cpp:202-222). Frames in flight
  // read version `cur` while an update writes the other one; a version is rewritten only after the launches
  // that read it (events per stream, ordered on the device).
  TlasVersion ver[2];
  int cur = -1;                  // the version launches read (-1: no TLAS)
  uint64_t blas_gen = 0;         // bumped by every BLAS build / rebuild
  uint64_t pool_gen = ~0ull;     // blas_gen the pool's BLAS part was laid out for
  uint32_t pool_tlas_cap = 0;    // nodes of each version's TLAS slot in the pool
  std::vector<uint32_t> node_base, tri_base;  // BLAS k's first node / triangle in the pools
  rt::BuildArena tlas_arena;     // lbvh_build scratch of the TLAS builds (kept: no hipMalloc per update)
  float* d_tlas_box = nullptr;   // instance world boxes (scratch, grown on demand)
  uint32_t tlas_scratch_cap = 0;
  double tlas_wall_ms = 0.0;     // host wall time of the last rt_tlas_build
  // frame state
  rt::FrameParams fp{};
  float cam_cb[64] = {};  // rt_set_camera's buffer: view, proj, viewInv, projInv in XMMATRIX memory order
  bool have_camera = false, have_shading = false;
  int schedule = RT_SCHED_PACKET;
  uint32_t tile_rows = 8;  // rt_set_tile_rows
  bool stats_on = false;
  unsigned long long* d_stats = nullptr;
  uint64_t dispatches = 0, pixels = 0;
  // row lists of strip dispatches (one slot per distinct list in use, keyed by content)
  ScratchRing rows;
  // traversal-stack overflow areas in HBM for lanes whose path outgrows the LDS part: one slot per
  // launch that may run concurrently with another (frames in flight, rt_trace_rays batches)
  ScratchRing ovf;
  // tile balance (rt_set_tile_balance): 0 off, 1 adaptive, 2 / 3 / 4 forced layouts (tests); one cost map per launch
  // shape (least recently used of kMaxBalanceMaps replaced); the work lists, one per launch in flight, from a ring
  int balance = 1;
  // the adaptive plan's split of costly tiles and its front class (PlanArgs::split, front; A/B diagnostics:
  // RT_BALANCE_SPLIT, RT_BALANCE_FRONT, RT_BALANCE_BUDGET — the extra waves as a divisor of the tiles — at context
  // creation) and the list's cover check (RT_BALANCE_CHECK, tests)
  uint32_t bal_split = 1, bal_front = 8, bal_check = 0, bal_budget = 8;
  uint32_t bal_forced_cap = 0;  // RT_BALANCE_FORCED_CAP (tests): the forced layouts' extra waves (0: 63 x the tiles)
  uint32_t bal_prio = 1;        // RT_BALANCE_PRIO (A/B): the front class's waves raise their issue priority
  uint32_t bal_fine = 1;        // RT_BALANCE_FINE (A/B): adaptive plans may split a tile into 64 one-pixel parts
  uint32_t bal_diag = 0;        // RT_BALANCE_DIAG (diagnostics: the recording kernel's traffic): 1 record
                                // on every launch and never use a list, 2 use the lists but stop recording once the
                                // first plan has started, 3 use the current list even where it does not pay
  static constexpr size_t kMaxBalanceMaps = 32;
  static constexpr uint32_t kRecycleBackoff = 16;
  std::vector<BalanceMap> bal;
  uint64_t bal_clock = 0;
  uint32_t bal_backoff = 0;  // launches of unknown shapes left before the next recycling scan
  BalanceMap* bal_last = nullptr;
  ScratchRing plans;
  // scene pools read by the trace kernels (rebuilt by every rt_tlas_build)
  rt::Bvh4Node* pool_nodes = nullptr;
  rt::TriRec* pool_tris = nullptr;
  size_t pool_nodes_cap = 0, pool_tris_cap = 0;
  bool tlas_stale = false;  // a BLAS was rebuilt after the last rt_tlas_build
  // raster fallback scratch (grown on demand)
  rt::RasterScratch raster;
  size_t raster_tile_cap = 0, raster_prim_cap = 0, raster_bin_cap = 0;
  uint32_t* raster_total_host = nullptr;  // pinned: the last draw's bin-entry total, copied back async
  rt::RasterDraws raster_draws_host;      // what raster.draws holds on the device (valid when n > 0)
  // every draw uses the one raster scratch: a draw on another stream waits (on the device) for the
  // previous draw, recorded here
  hipEvent_t raster_ev = nullptr;
  hipStream_t raster_stream = nullptr;
  bool raster_pending = false;
  uint64_t rows_gen = 0;  // row-list generations (ensure_rows uploads, rt_comm plans)
  // rt_ctx_counters: device-wide synchronisations (quiesce), balance maps recycled for a new shape, launches that ran
  // the plain grid because every map was in use
  uint64_t n_quiesce = 0, bal_recycled = 0, bal_full = 0;
  uint64_t bal_recycled_planned = 0;  // recycled maps that went on to start a plan (recycling that paid off)
};


namespace {

rt_status fail(rt_ctx* c, rt_status st, const std::string& msg) {
  if (c) c->err = msg;
  return st;
}

rt_status hip_fail(rt_ctx* c, hipError_t e, const char* what) {
  std::string m = std::string(what) + ": " + hipGetErrorString(e);
  return fail(c, e == hipErrorOutOfMemory ? RT_E_OOM : RT_E_HIP, m);
}

#define HIPCHK(ctx, x, what)                       \
  do {                                             \
    hipError_t e_ = (x);                           \
    if (e_ != hipSuccess) return hip_fail(ctx, e_, what); \
  } while (0)

// Waits for every launch that may still read the context's device buffers. Dispatches run on
// caller streams (rt_dispatch_rays / rt_trace_rays / rt_raster_draw take any hipStream_t), so a
// sync of the context's own stream is not enough before an in-place overwrite or a free: the
// reference waits on its fence the same way before it rebuilds (D3D12HelloTriangle.cpp:1482-1568).
// Only the rare mutating calls pay this (builds, rebuilds, a changed row list, buffer growth).
hipError_t quiesce(rt_ctx* c) {
  (void)hipSetDevice(c->device);
  ++c->n_quiesce;
  return hipDeviceSynchronize();
}

// Runs f on scope exit: frees a build's device scratch on every return path.
template <class F>
struct ScopeExit {
  F f;
  explicit ScopeExit(F fn) : f(fn) {}
  ~ScopeExit() { f(); }
  ScopeExit(const ScopeExit&) = delete;
  ScopeExit& operator=(const ScopeExit&) = delete;
};

// inverse of a 3x3 (row-major) in double, rounded to float; returns false if singular.
bool inverse3(const double m[9], double inv[9]) {
  double c00 = m[4] * m[8] - m[5] * m[7];
  double c01 = m[5] * m[6] - m[3] * m[8];
  double c02 = m[3] * m[7] - m[4] * m[6];
  double det = m[0] * c00 + m[1] * c01 + m[2] * c02;
  if (det == 0.0) return false;
  double r = 1.0 / det;
  inv[0] = c00 * r;
  inv[1] = (m[2] * m[7] - m[1] * m[8]) * r;
  inv[2] = (m[1] * m[5] - m[2] * m[4]) * r;
  inv[3] = c01 * r;
  inv[4] = (m[0] * m[8] - m[2] * m[6]) * r;
  inv[5] = (m[2] * m[3] - m[0] * m[5]) * r;
  inv[6] = c02 * r;
  inv[7] = (m[1] * m[6] - m[0] * m[7]) * r;
  inv[8] = (m[0] * m[4] - m[1] * m[3]) * r;
  return true;
}

// Fills the transform part of an InstanceRec (world-to-object, normal matrix) from a 3x4
// object-to-world transform. Same double-precision formulas as oracle/rt_oracle.c.
bool fill_instance_xform(const float* o2w, rt::InstanceRec& r) {
  double L[9] = {o2w[0], o2w[1], o2w[2], o2w[4], o2w[5], o2w[6], o2w[8], o2w[9], o2w[10]};
  double Li[9];
  if (!inverse3(L, Li)) return false;
  // winding sense for back-face culling: a mirroring transform swaps front and back
  const double det = L[0] * (L[4] * L[8] - L[5] * L[7]) + L[1] * (L[5] * L[6] - L[3] * L[8]) +
                     L[2] * (L[3] * L[7] - L[4] * L[6]);
  r.flip = det < 0.0 ? 1u : 0u;
  r.translate = (o2w[0] == 1.0f && o2w[1] == 0.0f && o2w[2] == 0.0f && o2w[4] == 0.0f && o2w[5] == 1.0f &&
               o2w[6] == 0.0f && o2w[8] == 0.0f && o2w[9] == 0.0f && o2w[10] == 1.0f) ? 1u : 0u;
  double t[3] = {o2w[3], o2w[7], o2w[11]};
  for (int i = 0; i < 3; ++i) {
    r.w2o[i * 4 + 0] = (float)Li[i * 3 + 0];
    r.w2o[i * 4 + 1] = (float)Li[i * 3 + 1];
    r.w2o[i * 4 + 2] = (float)Li[i * 3 + 2];
    r.w2o[i * 4 + 3] = (float)(-(Li[i * 3 + 0] * t[0] + Li[i * 3 + 1] * t[1] + Li[i * 3 + 2] * t[2]));
  }
  for (int i = 0; i < 12; ++i) r.o2w[i] = o2w[i];
  // objectToWorldNormal = transpose(inverse(upper3x3)) (D3D12HelloTriangle.cpp:1190-1200)
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) r.nrm[i * 3 + j] = (float)Li[j * 3 + i];
  return true;
}

rt_status upload_blas(rt_ctx* c, DeviceBlas& b, const void* vtx, uint32_t vcount, uint32_t stride,
                      const uint32_t* idx, uint32_t icount) {
  if (!vtx || vcount == 0 || stride < 12 || (stride % 4)) return fail(c, RT_E_INVALID, "rt_blas_build: bad vertex buffer");
  uint32_t ntri;
  if (idx) {
    if (icount == 0 || icount % 3) return fail(c, RT_E_INVALID, "rt_blas_build: index count must be a positive multiple of 3");
    for (uint32_t i = 0; i < icount; ++i)
      if (idx[i] >= vcount) return fail(c, RT_E_INVALID, "rt_blas_build: index out of range");
    ntri = icount / 3;
  } else {
    if (vcount % 3) return fail(c, RT_E_INVALID, "rt_blas_build: non-indexed vertex count must be a multiple of 3");
    ntri = vcount / 3;
  }
  // repack to {pos, normal} (normal default (0,1,0) when the stride carries none)
  std::vector<float> v6((size_t)vcount * 6);
  const unsigned char* src = (const unsigned char*)vtx;
  for (uint32_t i = 0; i < vcount; ++i) {
    const float* p = (const float*)(src + (size_t)i * stride);
    v6[i * 6 + 0] = p[0];
    v6[i * 6 + 1] = p[1];
    v6[i * 6 + 2] = p[2];
    if (stride >= 24) {
      v6[i * 6 + 3] = p[3];
      v6[i * 6 + 4] = p[4];
      v6[i * 6 + 5] = p[5];
    } else {
      v6[i * 6 + 3] = 0.0f;
      v6[i * 6 + 4] = 1.0f;
      v6[i * 6 + 5] = 0.0f;
    }
  }
  b.release();
  hipStream_t s = c->stream;
  HIPCHK(c, hipMalloc(&b.vtx, v6.size() * sizeof(float)), "hipMalloc(vtx)");
  HIPCHK(c, hipMemcpyAsync(b.vtx, v6.data(), v6.size() * sizeof(float), hipMemcpyHostToDevice, s), "upload vtx");
  if (idx) {
    HIPCHK(c, hipMalloc(&b.idx, (size_t)icount * 4), "hipMalloc(idx)");
    HIPCHK(c, hipMemcpyAsync(b.idx, idx, (size_t)icount * 4, hipMemcpyHostToDevice, s), "upload idx");
  }
  const uint32_t nn = ntri > 1 ? ntri - 1 : 1;
  rt::TriRec* unsorted = nullptr;
  float* primbox = nullptr;
  uint32_t* sorted = nullptr;
  auto free_fn = [&] {  // every return below (the caller releases b on failure)
    if (unsorted) (void)hipFree(unsorted);
    if (primbox) (void)hipFree(primbox);
    if (sorted) (void)hipFree(sorted);
  };
  ScopeExit<decltype(free_fn)> scratch(free_fn);
  HIPCHK(c, hipMalloc(&b.nodes, (size_t)nn * sizeof(rt::Bvh4Node)), "hipMalloc(nodes)");
  HIPCHK(c, hipMalloc(&b.tris, (size_t)ntri * sizeof(rt::TriRec)), "hipMalloc(tris)");
  HIPCHK(c, hipMalloc(&unsorted, (size_t)ntri * sizeof(rt::TriRec)), "hipMalloc(scratch)");
  HIPCHK(c, hipMalloc(&primbox, (size_t)ntri * 24), "hipMalloc(scratch)");
  HIPCHK(c, hipMalloc(&sorted, (size_t)ntri * 4), "hipMalloc(scratch)");
  hipError_t e = rt::blas_prepare(b.vtx, b.idx, ntri, unsorted, primbox, s);
  float ms = 0.0f;
  uint32_t nnodes4 = 0;
  if (e == hipSuccess)
    e = rt::lbvh_build(primbox, ntri, b.nodes, sorted, false, &nnodes4, &b.depth, &b.max_stack, b.bounds, &ms, s,
                       unsorted, b.tris);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hip_fail(c, e, "BLAS build");
  b.ntri = ntri;
  b.nnodes = nnodes4;
  b.nvtx = vcount;
  b.build_ms = ms;
  return RT_OK;
}

hipStream_t pick_stream(rt_ctx* c, void* s) { return s ? (hipStream_t)s : c->stream; }


}  // namespace

extern "C" {

int rt_api_version(void) { return RT_API_VERSION; }

const char* rt_status_string(rt_status st) {
  switch (st) {
    case RT_OK: return "RT_OK";
    case RT_E_INVALID: return "RT_E_INVALID";
    case RT_E_OOM: return "RT_E_OOM";
    case RT_E_HIP: return "RT_E_HIP";
    case RT_E_RCCL: return "RT_E_RCCL";
    case RT_E_UNSUPPORTED: return "RT_E_UNSUPPORTED";
    case RT_E_IO: return "RT_E_IO";
  }
  return "RT_E_UNKNOWN";
}

const char* rt_last_error(rt_ctx_t ctx) { return ctx ? ctx->err.c_str() : "null context"; }

rt_status rt_create(int hip_device, rt_ctx_t* out) {
  if (!out) return RT_E_INVALID;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return RT_E_UNSUPPORTED;
  if (hip_device < 0 || hip_device >= n) return RT_E_INVALID;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, hip_device) != hipSuccess) return RT_E_HIP;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return RT_E_UNSUPPORTED;
  if (hipSetDevice(hip_device) != hipSuccess) return RT_E_HIP;
  rt_ctx* c = new (std::nothrow) rt_ctx();
  if (!c) return RT_E_OOM;
  c->device = hip_device;
  if (const char* ev = std::getenv("RT_BALANCE_SPLIT")) c->bal_split = std::strtoul(ev, nullptr, 10) ? 1u : 0u;
  if (const char* ev = std::getenv("RT_BALANCE_DIAG")) c->bal_diag = (uint32_t)std::strtoul(ev, nullptr, 10);
  if (const char* ev = std::getenv("RT_BALANCE_FRONT")) c->bal_front = (uint32_t)std::strtoul(ev, nullptr, 10);
  if (const char* ev = std::getenv("RT_BALANCE_CHECK")) c->bal_check = std::strtoul(ev, nullptr, 10) ? 1u : 0u;
  if (const char* ev = std::getenv("RT_BALANCE_BUDGET"))
    c->bal_budget = std::max<uint32_t>(1u, (uint32_t)std::strtoul(ev, nullptr, 10));
  if (const char* ev = std::getenv("RT_BALANCE_PRIO")) c->bal_prio = std::strtoul(ev, nullptr, 10) ? 1u : 0u;
  if (const char* ev = std::getenv("RT_BALANCE_FINE")) c->bal_fine = std::strtoul(ev, nullptr, 10) ? 1u : 0u;
  if (const char* ev = std::getenv("RT_BALANCE_FORCED_CAP")) c->bal_forced_cap = (uint32_t)std::strtoul(ev, nullptr, 10);
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&c->d_stats, RT_STAT_COUNT * sizeof(unsigned long long)) != hipSuccess ||
      hipMemset(c->d_stats, 0, RT_STAT_COUNT * sizeof(unsigned long long)) != hipSuccess) {
    delete c;
    return RT_E_HIP;
  }
  *out = c;
  return RT_OK;
}

rt_status rt_destroy(rt_ctx_t c) {
  if (!c) return RT_E_INVALID;
  (void)hipSetDevice(c->device);
  (void)quiesce(c);  // launches on caller streams may still read the context's buffers
  for (auto& b : c->blas) b.release();
  for (auto& v : c->ver) v.release();
  c->tlas_arena.release();
  if (c->d_tlas_box) (void)hipFree(c->d_tlas_box);
  if (c->d_stats) (void)hipFree(c->d_stats);
  for (auto& sl : c->rows.slots) slot_release(sl);
  for (auto& sl : c->ovf.slots) slot_release(sl);
  for (auto& sl : c->plans.slots) slot_release(sl);
  for (auto& m : c->bal) m.release();
  if (c->raster_ev) (void)hipEventDestroy(c->raster_ev);
  if (c->pool_nodes) (void)hipFree(c->pool_nodes);
  if (c->pool_tris) (void)hipFree(c->pool_tris);
  for (void* p : {(void*)c->raster.clip, (void*)c->raster.slots, (void*)c->raster.tiles, (void*)c->raster.tcount,
                  (void*)c->raster.toffs, (void*)c->raster.bins, (void*)c->raster.bsum, (void*)c->raster.draws})
    if (p) (void)hipFree(p);
  if (c->raster_total_host) (void)hipHostFree(c->raster_total_host);
  (void)hipStreamDestroy(c->stream);
  delete c;
  return RT_OK;
}

rt_status rt_blas_build(rt_ctx_t c, const void* vtx, uint32_t vcount, uint32_t stride,
                        const uint32_t* idx, uint32_t icount, rt_blas_t* out) {
  if (!c || !out) return fail(c, RT_E_INVALID, "rt_blas_build: null argument");
  (void)hipSetDevice(c->device);
  DeviceBlas b;
  rt_status st = upload_blas(c, b, vtx, vcount, stride, idx, icount);
  if (st != RT_OK) {
    b.release();
    return st;
  }
  c->blas.push_back(b);
  ++c->blas_gen;
  *out = (rt_blas_t)(c->blas.size() - 1);
  return RT_OK;
}

rt_status rt_blas_rebuild(rt_ctx_t c, rt_blas_t id, const void* vtx, uint32_t vcount, uint32_t stride,
                          const uint32_t* idx, uint32_t icount) {
  if (!c || id >= c->blas.size()) return fail(c, RT_E_INVALID, "rt_blas_rebuild: unknown BLAS");
  // frames in flight on any stream shade from this BLAS's vertex / index arrays
  HIPCHK(c, quiesce(c), "rt_blas_rebuild: wait for in-flight work");
  DeviceBlas b;
  rt_status st = upload_blas(c, b, vtx, vcount, stride, idx, icount);
  if (st != RT_OK) {
    b.release();
    return st;
  }
  c->blas[id].release();
  c->blas[id] = b;
  ++c->blas_gen;
  c->tlas_stale = c->cur >= 0;  // the scene pool holds the old tree until rt_tlas_build
  return RT_OK;
}

rt_status rt_blas_info(rt_ctx_t c, rt_blas_t id, rt_bvh_info* out) {
  if (!c || !out || id >= c->blas.size()) return fail(c, RT_E_INVALID, "rt_blas_info: bad argument");
  const DeviceBlas& b = c->blas[id];
  out->prim_count = b.ntri;
  out->node_count = b.nnodes;
  out->depth = b.depth;
  out->max_stack = b.max_stack;
  for (int k = 0; k < 3; ++k) {
    out->bounds_lo[k] = b.bounds[k];
    out->bounds_hi[k] = b.bounds[3 + k];
  }
  out->build_ms = b.build_ms;
  return RT_OK;
}

rt_status rt_blas_export(rt_ctx_t c, rt_blas_t id, void* nodes, size_t nodes_bytes, void* tris,
                         size_t tris_bytes) {
  if (!c || id >= c->blas.size()) return fail(c, RT_E_INVALID, "rt_blas_export: unknown BLAS");
  const DeviceBlas& b = c->blas[id];
  (void)hipSetDevice(c->device);
  if (nodes) {
    if (nodes_bytes < (size_t)b.nnodes * sizeof(rt::Bvh4Node))
      return fail(c, RT_E_INVALID, "rt_blas_export: nodes buffer too small");
    HIPCHK(c, hipMemcpy(nodes, b.nodes, (size_t)b.nnodes * sizeof(rt::Bvh4Node), hipMemcpyDeviceToHost), "export nodes");
  }
  if (tris) {
    if (tris_bytes < (size_t)b.ntri * 48) return fail(c, RT_E_INVALID, "rt_blas_export: tris buffer too small");
    HIPCHK(c, hipMemcpy(tris, b.tris, (size_t)b.ntri * 48, hipMemcpyDeviceToHost), "export tris");
  }
  return RT_OK;
}

rt_status rt_tlas_build(rt_ctx_t c, const rt_instance* in, uint32_t n, int update_only) {
  if (!c || !in || n == 0) return fail(c, RT_E_INVALID, "rt_tlas_build: need at least one instance");
  const auto t_start = std::chrono::steady_clock::now();
  (void)hipSetDevice(c->device);
  if (update_only) {
    const TlasVersion* cv = c->cur >= 0 ? &c->ver[c->cur] : nullptr;
    if (!cv || c->tlas_stale || n != cv->ninst)
      return fail(c, RT_E_INVALID, "rt_tlas_build: update needs the same instance count");
    for (uint32_t i = 0; i < n; ++i)
      if (in[i].blas != cv->host[i].blas) return fail(c, RT_E_INVALID, "rt_tlas_build: update cannot change BLAS");
  }
  std::vector<rt::InstanceRec> recs(n);
  std::vector<float> bb((size_t)n * 6);
  for (uint32_t i = 0; i < n; ++i) {
    if (in[i].blas >= c->blas.size()) return fail(c, RT_E_INVALID, "rt_tlas_build: unknown BLAS id");
    if (in[i].hit_group != RT_HITGROUP_MODEL && in[i].hit_group != RT_HITGROUP_PLANE)
      return fail(c, RT_E_INVALID, "rt_tlas_build: hit_group must be 0 (model) or 2 (plane)");
    rt::InstanceRec& r = recs[i];
    std::memset(&r, 0, sizeof(r));
    if (!fill_instance_xform(in[i].xform3x4_rowmajor, r)) return fail(c, RT_E_INVALID, "rt_tlas_build: singular transform");
    const DeviceBlas& b = c->blas[in[i].blas];
    r.instance_id = in[i].instance_id;
    r.hit_group = in[i].hit_group;
    r.blas = in[i].blas;
    r.nodes = b.nodes;
    r.tris = b.tris;
    r.vtx = b.vtx;
    r.idx = b.idx;
    for (int k = 0; k < 6; ++k) bb[i * 6 + k] = b.bounds[k];
  }
  const uint32_t tlas_cap = n > 1 ? n - 1 : 1;
  hipStream_t s = c->stream;
  // Fast path (a per-frame update): the pool's BLAS part is current and each version's arrays and pool slot
  // hold n instances. The version launches do not read is written after ITS last launches (device-side waits),
  // with scratch kept from earlier builds: no device-wide synchronisation, no allocation. The host waits for
  // this build alone (the tree's node count and stack bound come back to size the next launches).
  const bool fast = c->pool_gen == c->blas_gen && c->pool_tlas_cap >= tlas_cap && c->ver[0].cap >= n &&
                    c->ver[1].cap >= n && c->tlas_scratch_cap >= n;
  if (!fast) {
    // layout change (BLAS built or rebuilt, more instances): every launch that may read the pools or the
    // instance records finishes first, as the reference waits on its fence before rebuilding (:1482-1568)
    HIPCHK(c, quiesce(c), "rt_tlas_build: wait for in-flight work");
    c->tlas_stale = true;  // until this build completes (a failure below leaves the scene unusable)
    c->cur = -1;
    c->ver[0].readers.clear();  // every launch has completed
    c->ver[1].readers.clear();
    size_t pool_n = 0, pool_t = 0;
    c->node_base.assign(c->blas.size(), 0);
    c->tri_base.assign(c->blas.size(), 0);
    for (size_t k = 0; k < c->blas.size(); ++k) {
      c->node_base[k] = (uint32_t)pool_n;
      c->tri_base[k] = (uint32_t)pool_t;
      pool_n += c->blas[k].nnodes;
      pool_t += c->blas[k].ntri;
    }
    const uint32_t slot_cap = std::max(tlas_cap, c->pool_tlas_cap);
    const size_t tlas0 = pool_n;
    pool_n += 2 * (size_t)slot_cap;
    if (pool_n > 0x7fffffffull / sizeof(rt::Bvh4Node) || pool_t > 0x7fffffffull / sizeof(rt::TriRec))
      return fail(c, RT_E_UNSUPPORTED, "rt_tlas_build: scene pool exceeds 2 GB of nodes or triangles");
    if (pool_n > c->pool_nodes_cap) {
      if (c->pool_nodes) (void)hipFree(c->pool_nodes);
      c->pool_nodes = nullptr;
      c->pool_nodes_cap = 0;
      HIPCHK(c, hipMalloc(&c->pool_nodes, pool_n * sizeof(rt::Bvh4Node)), "hipMalloc(node pool)");
      c->pool_nodes_cap = pool_n;
    }
    if (pool_t > c->pool_tris_cap) {
      if (c->pool_tris) (void)hipFree(c->pool_tris);
      c->pool_tris = nullptr;
      c->pool_tris_cap = 0;
      HIPCHK(c, hipMalloc(&c->pool_tris, pool_t * sizeof(rt::TriRec)), "hipMalloc(triangle pool)");
      c->pool_tris_cap = pool_t;
    }
    hipError_t e = hipSuccess;
    for (size_t k = 0; k < c->blas.size() && e == hipSuccess; ++k) {  // the BLAS part: once per layout
      const DeviceBlas& b = c->blas[k];
      e = rt::pool_rebase(b.nodes, b.nnodes, c->node_base[k], c->tri_base[k], c->pool_nodes + c->node_base[k], s);
      if (e == hipSuccess)
        e = hipMemcpyAsync(c->pool_tris + c->tri_base[k], b.tris, (size_t)b.ntri * sizeof(rt::TriRec),
                           hipMemcpyDeviceToDevice, s);
    }
    if (e != hipSuccess) return hip_fail(c, e, "scene pool");
    for (int v = 0; v < 2; ++v) {
      TlasVersion& tv = c->ver[v];
      tv.valid = false;
      tv.pool_base = (uint32_t)(tlas0 + (size_t)v * slot_cap);
      if (tv.cap < n) {
        if (tv.nodes) (void)hipFree(tv.nodes);
        if (tv.inst) (void)hipFree(tv.inst);
        if (tv.sorted) (void)hipFree(tv.sorted);
        if (tv.staging) (void)hipHostFree(tv.staging);
        tv.nodes = nullptr;
        tv.inst = nullptr;
        tv.sorted = nullptr;
        tv.staging = nullptr;
        tv.cap = 0;
        HIPCHK(c, hipMalloc(&tv.nodes, (size_t)tlas_cap * sizeof(rt::Bvh4Node)), "hipMalloc(tlas)");
        // the instance records, then the BLAS boxes of the build (one upload from the staging, same layout)
        HIPCHK(c, hipMalloc(&tv.inst, (size_t)n * (sizeof(rt::InstanceRec) + 24)), "hipMalloc(instances)");
        HIPCHK(c, hipMalloc(&tv.sorted, (size_t)n * 4), "hipMalloc(tlas order)");
        tv.staging_bytes = (size_t)n * sizeof(rt::InstanceRec) + (size_t)n * 24;
        HIPCHK(c, hipHostMalloc((void**)&tv.staging, tv.staging_bytes, hipHostMallocDefault), "hipHostMalloc(tlas staging)");
        tv.cap = n;
      }
      if (!tv.ready && !(tv.ready = new_sync_event())) return fail(c, RT_E_HIP, "rt_tlas_build: event");
    }
    if (c->tlas_scratch_cap < n) {
      if (c->d_tlas_box) (void)hipFree(c->d_tlas_box);
      c->d_tlas_box = nullptr;
      c->tlas_scratch_cap = 0;
      HIPCHK(c, hipMalloc(&c->d_tlas_box, (size_t)n * 24), "hipMalloc(tlas scratch)");
      c->tlas_scratch_cap = n;
    }
    c->pool_tlas_cap = slot_cap;
    c->pool_gen = c->blas_gen;
  }
  // the version launches do not read now
  const int w = c->cur >= 0 ? 1 - c->cur : 0;
  TlasVersion& tv = c->ver[w];
  for (uint32_t i = 0; i < n; ++i) recs[i].pool_root = c->node_base[recs[i].blas];
  // its previous readers on other streams finish before the upload overwrites it (device-side waits)
  HIPCHK(c, slot_order_after_others(tv.use, s), "rt_tlas_build: order after the version's launches");
  std::memcpy(tv.staging, recs.data(), recs.size() * sizeof(rt::InstanceRec));  // staging idle: its last build synced
  float* bb_stage = (float*)((char*)tv.staging + (size_t)n * sizeof(rt::InstanceRec));
  std::memcpy(bb_stage, bb.data(), bb.size() * 4);
  // records and boxes in one copy: the version's buffer holds the n records, then the n BLAS boxes
  const float* d_bb = (const float*)((const char*)tv.inst + (size_t)n * sizeof(rt::InstanceRec));
  hipError_t e = hipMemcpyAsync(tv.inst, tv.staging, (size_t)n * sizeof(rt::InstanceRec) + bb.size() * 4,
                                hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = rt::tlas_prepare(tv.inst, d_bb, n, c->d_tlas_box, s);
  float ms = 0.0f;
  uint32_t nn = 0, depth = 0, mstack = 0;
  float bounds[6];
  // update_only rebuilds the hierarchy over the new boxes: an LBVH rebuild costs the same launches as a
  // refit at these sizes and keeps the tree identical to a fresh build
  if (e == hipSuccess)
    e = rt::lbvh_build(c->d_tlas_box, n, tv.nodes, tv.sorted, true, &nn, &depth, &mstack, bounds, &ms, s, nullptr,
                       nullptr, &c->tlas_arena);
  if (e == hipSuccess) e = rt::pool_rebase(tv.nodes, nn, tv.pool_base, -1, c->pool_nodes + tv.pool_base, s);
  if (e == hipSuccess) e = hipEventRecord(tv.ready, s);
  if (e != hipSuccess) {
    tv.valid = false;
    return hip_fail(c, e, "TLAS build");
  }
  tv.ready_pending = true;
  tv.ninst = n;
  tv.nodes_n = nn;
  tv.depth = depth;
  tv.max_stack = mstack;
  std::memcpy(tv.bounds, bounds, sizeof(bounds));
  tv.ms = ms;
  tv.host.assign(in, in + n);
  tv.valid = true;
  // the version launches read until now: its readers' events, recorded now, cover every launch that read it
  if (c->cur >= 0 && c->cur != w) HIPCHK(c, note_swap_out(c->ver[c->cur]), "rt_tlas_build: record the readers");
  c->cur = w;
  c->tlas_stale = false;
  c->tlas_wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
  return RT_OK;
}

rt_status rt_tlas_info(rt_ctx_t c, rt_bvh_info* out) {
  if (!c || !out || c->cur < 0) return fail(c, RT_E_INVALID, "rt_tlas_info: no TLAS");
  const TlasVersion& v = c->ver[c->cur];
  out->prim_count = v.ninst;
  out->node_count = v.nodes_n;
  out->depth = v.depth;
  out->max_stack = v.max_stack;
  for (int k = 0; k < 3; ++k) {
    out->bounds_lo[k] = v.bounds[k];
    out->bounds_hi[k] = v.bounds[3 + k];
  }
  out->build_ms = v.ms;
  return RT_OK;
}

double rt_tlas_build_wall_ms(rt_ctx_t c) { return c ? c->tlas_wall_ms : 0.0; }

rt_status rt_tlas_export(rt_ctx_t c, void* nodes, size_t nodes_bytes) {
  if (!c || !nodes || c->cur < 0) return fail(c, RT_E_INVALID, "rt_tlas_export: no TLAS");
  const TlasVersion& v = c->ver[c->cur];
  const size_t bytes = (size_t)v.nodes_n * sizeof(rt::Bvh4Node);
  if (nodes_bytes < bytes) return fail(c, RT_E_INVALID, "rt_tlas_export: buffer too small");
  (void)hipSetDevice(c->device);
  HIPCHK(c, hipMemcpy(nodes, v.nodes, bytes, hipMemcpyDeviceToHost), "export tlas");
  return RT_OK;
}

rt_status rt_set_camera(rt_ctx_t c, const float cb[64]) {
  if (!c || !cb) return fail(c, RT_E_INVALID, "rt_set_camera: null argument");
  std::memcpy(c->cam_cb, cb, 64 * sizeof(float));  // RayGen's constants are derived per launch (frame_cam)
  c->have_camera = true;
  return RT_OK;
}

rt_status rt_set_shading(rt_ctx_t c, const rt_light* lights, uint32_t nlights, const rt_material* m,
                         int shade_mode, int spp) {
  if (!c || !lights || !m) return fail(c, RT_E_INVALID, "rt_set_shading: null argument");
  if (nlights < 1 || nlights > (uint32_t)rt::kMaxLights) return fail(c, RT_E_INVALID, "rt_set_shading: nlights must be in [1,16]");
  if (shade_mode < RT_SHADE_REF || shade_mode > RT_SHADE_PRIMARY) return fail(c, RT_E_INVALID, "rt_set_shading: unknown shade mode");
  int k = 0;
  for (int s = 1; s <= 4; ++s)
    if (s * s == spp) k = s;
  if (!k) return fail(c, RT_E_INVALID, "rt_set_shading: spp must be 1, 4, 9 or 16");
  for (uint32_t l = 0; l < nlights; ++l) std::memcpy(&c->fp.lights[l], &lights[l], sizeof(rt::LightRec));
  std::memcpy(&c->fp.material, m, sizeof(rt::MaterialRec));
  rt::surface_consts(c->fp.material, c->fp.surf);
  c->fp.nlights = nlights;
  c->fp.shade_mode = (uint32_t)shade_mode;
  c->fp.spp_side = (uint32_t)k;
  c->have_shading = true;
  return RT_OK;
}

rt_status rt_set_schedule(rt_ctx_t c, int schedule) {
  if (!c) return RT_E_INVALID;
  if (schedule != RT_SCHED_PACKET && schedule != RT_SCHED_LANE) return fail(c, RT_E_INVALID, "rt_set_schedule: unknown schedule");
  c->schedule = schedule;
  return RT_OK;
}

rt_status rt_set_tile_rows(rt_ctx_t c, int rows) {
  if (!c) return RT_E_INVALID;
  if (rows != 4 && rows != 8) return fail(c, RT_E_INVALID, "rt_set_tile_rows: rows must be 4 or 8");
  c->tile_rows = (uint32_t)rows;
  return RT_OK;
}

rt_status rt_set_tile_balance(rt_ctx_t c, int mode) {
  if (!c) return RT_E_INVALID;
  if (mode < 0 || mode > 5) return fail(c, RT_E_INVALID, "rt_set_tile_balance: mode 0 .. 5");
  c->balance = mode;
  return RT_OK;
}

rt_status rt_ctx_counters_n(rt_ctx_t c, uint64_t* out, uint32_t n) {
  if (!c || (!out && n)) return RT_E_INVALID;
  const uint64_t v[RT_CTX_COUNTERS_V2] = {c->n_quiesce, c->bal_recycled, c->bal_full, c->bal.size(),
                                          c->bal_recycled_planned};
  std::memcpy(out, v, std::min<uint32_t>(n, RT_CTX_COUNTERS_V2) * sizeof(uint64_t));
  return RT_OK;
}

rt_status rt_ctx_counters(rt_ctx_t c, uint64_t out[RT_CTX_COUNTERS]) { return rt_ctx_counters_n(c, out, RT_CTX_COUNTERS); }

rt_status rt_tile_balance_info_n(rt_ctx_t c, uint32_t* out_words, uint32_t n) {
  if (!c || (!out_words && n)) return RT_E_INVALID;
  uint32_t out[RT_BALANCE_INFO_COUNT];
  std::memset(out, 0, sizeof(out));
  std::memset(out_words, 0, std::min<uint32_t>(n, RT_BALANCE_INFO_COUNT) * sizeof(uint32_t));
  const BalanceMap* m = c->bal_last;
  if (!m || !m->stats) return RT_OK;
  const volatile rt::PlanStats* st = m->stats;
  out[0] = st->plans;
  out[1] = st->nsplit;
  out[2] = st->nitems;
  out[3] = m->extra_cap;
  out[4] = st->max_cost;
  out[5] = st->mean_cost;
  out[6] = st->threshold;
  out[7] = (uint32_t)std::min<uint64_t>(m->launches, 0xffffffffu);
  out[8] = st->pays;
  out[9] = st->bad;
  out[10] = st->first_bad_tile;
  out[11] = st->first_bad_word;
  for (int k = 0; k < 3; ++k) out[12 + k] = st->phase_ticks[k];
  out[15] = st->slots;
  out[16] = st->refused;
  out[17] = st->refused_plans;
  std::memcpy(out_words, out, std::min<uint32_t>(n, RT_BALANCE_INFO_COUNT) * sizeof(uint32_t));
  return RT_OK;
}

// the round-4 entry point: exactly its 16 words (a caller built against uint32_t[16] must not be overrun)
rt_status rt_tile_balance_info(rt_ctx_t c, uint32_t out[RT_BALANCE_INFO_COUNT_V1]) {
  return rt_tile_balance_info_n(c, out, RT_BALANCE_INFO_COUNT_V1);
}

rt_status rt_set_stats(rt_ctx_t c, int enable) {
  if (!c) return RT_E_INVALID;
  c->stats_on = enable != 0;
  return RT_OK;
}

static rt::SceneView scene_view(rt_ctx* c) {
  rt::SceneView sv;
  const TlasVersion& v = c->ver[c->cur];
  sv.pool_nodes = c->pool_nodes;
  sv.pool_tris = c->pool_tris;
  sv.tlas = v.nodes;
  sv.inst = v.inst;
  sv.tlas_root = (int)v.pool_base;
  uint32_t maxb = 0, maxd = 0;
  for (const auto& b : c->blas) {
    maxb = b.max_stack > maxb ? b.max_stack : maxb;
    maxd = b.depth > maxd ? b.depth : maxd;
  }
  // worst case: the TLAS path's siblings, the TLAS->BLAS sentinel, the BLAS path's siblings
  sv.stack_cap = (int)(v.max_stack + 1 + maxb);
  // wave packets: the TLAS path's siblings, then at most one entry per BLAS level
  sv.packet_cap = (int)(v.max_stack + maxd);
  sv.lds_cap = sv.stack_cap < rt::kLdsStackEntries ? sv.stack_cap : rt::kLdsStackEntries;
  sv.ovf = nullptr;
  sv.ovf_lanes = 0;
  sv.cull_sense = 1.0f;
  sv.hybrid = maxb <= (uint32_t)rt::kHybridStack ? 1 : 0;
#if RT_LDS_TOP
  sv.lds_root = 0;
  sv.lds_n = 0;
  for (size_t k = 0; k < c->blas.size() && k < c->node_base.size(); ++k)
    if ((int)c->blas[k].nnodes > sv.lds_n) {
      sv.lds_n = (int)c->blas[k].nnodes;
      sv.lds_root = (int)c->node_base[k];
    }
  sv.lds_n = sv.lds_n < RT_LDS_TOP ? sv.lds_n : RT_LDS_TOP;
#endif
  return sv;
}

// A launch on s reads the current TLAS version: it waits (on the device) for that version's build, enqueued
// on the context stream, unless s is that stream or the build is seen complete.
static hipError_t order_after_tlas(rt_ctx* c, hipStream_t s) {
  TlasVersion& v = c->ver[c->cur];
  if (!v.ready_pending || s == c->stream) return hipSuccess;
  if (hipEventQuery(v.ready) == hipSuccess) {
    v.ready_pending = false;
    return hipSuccess;
  }
  return hipStreamWaitEvent(s, v.ready, 0);
}

// Picks the ring slot a launch on s uses (see ScratchRing). `match` (row lists): a slot holding
// the same content is shared as is — launches only read it.
static ScratchSlot* ring_acquire(ScratchRing& ring, hipStream_t s, const std::vector<uint32_t>* match, bool* hit,
                                 hipError_t* err) {
  *hit = false;
  *err = hipSuccess;
  ScratchSlot* pick = nullptr;
  if (match) {
    for (ScratchSlot& sl : ring.slots)
      if (sl.key == *match) {
        *hit = true;
        sl.tick = ++ring.clock;
        return &sl;
      }
  }
  for (ScratchSlot& sl : ring.slots)  // idle for s: only s used it, or every other use completed
    if (slot_free_for(sl, s) && (!pick || sl.tick < pick->tick)) pick = &sl;
  if (!pick && ring.slots.size() < ScratchRing::kMaxSlots) {
    ring.slots.emplace_back();
    pick = &ring.slots.back();
  }
  if (!pick) {  // every slot busy on other streams: the least recently used one, ordered on the device
    for (ScratchSlot& sl : ring.slots)
      if (!pick || sl.tick < pick->tick) pick = &sl;
    *err = slot_order_after_others(*pick, s);
  }
  pick->tick = ++ring.clock;
  return pick;
}

// grows a slot's device buffer (the host waits for the slot's own uses, not the whole device)
static hipError_t slot_reserve(ScratchSlot& sl, size_t bytes) {
  if (sl.cap >= bytes) return hipSuccess;
  hipError_t e = slot_drain(sl);
  if (e != hipSuccess) return e;
  if (sl.buf) (void)hipFree(sl.buf);
  sl.buf = nullptr;
  sl.cap = 0;
  e = hipMalloc(&sl.buf, bytes);
  if (e == hipSuccess) sl.cap = bytes;
  return e;
}

// The HBM overflow stack for `lanes` lanes when the trees are deeper than the LDS part: a slot of
// its own per concurrent launch. Returns the slot to mark after the launch (nullptr: none needed).
static rt_status ensure_overflow(rt_ctx* c, rt::SceneView& sv, size_t lanes, hipStream_t s, ScratchSlot** used) {
  *used = nullptr;
  if (sv.stack_cap <= sv.lds_cap) return RT_OK;
  const size_t need = lanes * (size_t)(sv.stack_cap - sv.lds_cap) * sizeof(int);
  bool hit;
  hipError_t e;
  ScratchSlot* sl = ring_acquire(c->ovf, s, nullptr, &hit, &e);
  if (e != hipSuccess) return hip_fail(c, e, "overflow stack: order after in-flight launches");
  HIPCHK(c, slot_reserve(*sl, need), "hipMalloc(stack overflow area)");
  sv.ovf = (int*)sl->buf;
  sv.ovf_lanes = (uint32_t)lanes;
  *used = sl;
  return RT_OK;
}

// Device copy of a strip dispatch's row list, shared by every launch that renders the same rows.
static rt_status ensure_rows(rt_ctx* c, const uint32_t* rows, uint32_t nrows, hipStream_t s, ScratchSlot** used,
                             const uint32_t** d_rows, uint64_t* gen) {
  std::vector<uint32_t> key(rows, rows + nrows);
  bool hit;
  hipError_t e;
  ScratchSlot* sl = ring_acquire(c->rows, s, &key, &hit, &e);
  if (e != hipSuccess) return hip_fail(c, e, "rows: order after in-flight launches");
  if (!hit) {
    const size_t bytes = (size_t)nrows * 4;
    HIPCHK(c, slot_reserve(*sl, bytes), "hipMalloc(rows)");
    // this slot held another list: every launch that read it (any stream) precedes the upload
    HIPCHK(c, slot_order_after_others(*sl, s), "rows: order after in-flight launches");
    if (sl->upload_ev && sl->uploaded) HIPCHK(c, hipEventSynchronize(sl->upload_ev), "rows staging");
    if (sl->staging_cap < bytes) {
      if (sl->staging) (void)hipHostFree(sl->staging);
      sl->staging = nullptr;
      sl->staging_cap = 0;
      HIPCHK(c, hipHostMalloc((void**)&sl->staging, bytes, hipHostMallocDefault), "hipHostMalloc(rows staging)");
      sl->staging_cap = bytes;
    }
    if (!sl->upload_ev && !(sl->upload_ev = new_sync_event())) return fail(c, RT_E_HIP, "rows: event");
    std::memcpy(sl->staging, rows, bytes);
    sl->key.swap(key);
    sl->gen = ++c->rows_gen;
    HIPCHK(c, hipMemcpyAsync(sl->buf, sl->staging, bytes, hipMemcpyHostToDevice, s), "upload rows");
    HIPCHK(c, hipEventRecord(sl->upload_ev, s), "upload rows");
    sl->uploaded = true;
    sl->upload_stream = s;
  } else if (sl->uploaded && sl->upload_stream != s) {
    // the same list, uploaded on another stream: this launch must not read it before the copy lands
    if (hipEventQuery(sl->upload_ev) == hipSuccess) sl->uploaded = false;  // landed: no wait from now on
    else HIPCHK(c, hipStreamWaitEvent(s, sl->upload_ev, 0), "rows: order after upload");
  }
  *used = sl;
  *d_rows = (const uint32_t*)sl->buf;
  *gen = sl->gen;
  return RT_OK;
}

}  // extern "C"

namespace rt {

int ctx_device(rt_ctx* c) { return c ? c->device : 0; }
uint64_t ctx_next_rows_gen(rt_ctx* c) { return c ? ++c->rows_gen : 0; }

hipError_t ctx_forget_stream(rt_ctx* c, hipStream_t s) {
  if (!c || !s) return hipSuccess;
  hipError_t first = hipSuccess;
  for (TlasVersion& v : c->ver) {
    auto it = std::find(v.readers.begin(), v.readers.end(), s);
    if (it == v.readers.end()) continue;
    v.readers.erase(it);
    const hipError_t e = slot_mark_use(v.use, s);  // covers every launch of s so far
    if (e != hipSuccess && first == hipSuccess) first = e;
  }
  // the tile balance's lists: the same for their readers
  for (BalanceMap& m : c->bal) {
    if (m.last_stream == s) m.last_stream = nullptr;
    auto used = std::find(m.streams.begin(), m.streams.end(), s);
    if (used != m.streams.end()) {
      // its last launch may still write the cost map: balance_idle queries this event before the map is recycled
      // (a recycled map's memset and new shape must not race a forgotten stream's cost stores)
      m.streams.erase(used);
      const hipError_t e = slot_mark_use(m.forgotten, s);
      if (e != hipSuccess && first == hipSuccess) first = e;
    }
    auto it = std::find(m.readers.begin(), m.readers.end(), s);
    if (it == m.readers.end() || m.cur < 0) continue;
    m.readers.erase(it);
    const hipError_t e = slot_mark_use(m.list[m.cur], s);
    if (e != hipSuccess && first == hipSuccess) first = e;
  }
  return first;
}
void* ctx_stream(rt_ctx* c) { return c ? (void*)c->stream : nullptr; }

rt_status check_dispatch(rt_ctx* c, uint32_t W, uint32_t H, const void* rgba8, bool cameras_given) {
  if (c->cur < 0 && !c->tlas_stale) return fail(c, RT_E_INVALID, "rt_dispatch_rays: no TLAS built");
  if (c->tlas_stale)
    return fail(c, RT_E_INVALID, "rt_dispatch_rays: scene stale (BLAS rebuilt, or the last rt_tlas_build failed)");
  if (!c->have_shading) return fail(c, RT_E_INVALID, "rt_dispatch_rays: shading not set");
  if (!c->have_camera && !cameras_given) return fail(c, RT_E_INVALID, "rt_dispatch_rays: camera not set");
  if (W == 0 || H == 0 || !rgba8) return fail(c, RT_E_INVALID, "rt_dispatch_rays: bad size or output");
  return RT_OK;
}

// Whether nothing in flight can touch a map's buffers any more: every stream that launched with it is idle and its
// pending plan (context stream) has completed. Host queries only (no device-wide synchronisation).
static bool balance_idle(const BalanceMap& m) {
  if (m.pending >= 0 && m.pend_ev && hipEventQuery(m.pend_ev) != hipSuccess) return false;
  for (hipStream_t s : m.streams)
    if (hipStreamQuery(s) != hipSuccess) return false;
  return slot_free_for(m.forgotten, nullptr);  // the forgotten streams' last launches too
}

// The load bound's wave slots for a plan: the occupancy of the kernel the list will drive (from the runtime, for
// the instantiation launched) x the device's CUs; the documented 8 waves per SIMD x 1024 SIMDs if the runtime
// cannot tell.
static uint32_t plan_slots(rt_ctx* c, const rt::SceneView& sv) {
  const uint32_t n = rt::trace_wave_slots(sv, c->fp, c->schedule, c->device);
  return n ? n : 8u * 1024u;
}

// The cost map of a launch shape (created with zero costs on stream s: the first launch runs the plain grid). With
// every map in use (kMaxBalanceMaps shapes: a loopback communicator emulating many ranks has one per rank), a map
// whose buffers nothing in flight can touch and whose cost buffer is large enough is recycled (never a
// device-wide synchronisation on the frame path); if there is none, null with *err = hipSuccess: the launch runs
// the plain grid. Forced layouts (tests) instead wait for the device and replace the least recently used map.
static BalanceMap* balance_map(rt_ctx* c, uint32_t W, uint32_t nrows, const uint32_t* d_rows, uint64_t rows_gen,
                               uint32_t nframes, uint32_t ntiles, hipStream_t s, bool forced, hipError_t* err) {
  *err = hipSuccess;
  BalanceMap* lru = nullptr;
  for (BalanceMap& m : c->bal) {
    if (m.W == W && m.nrows == nrows && m.rows == d_rows && m.rows_gen == rows_gen && m.nframes == nframes &&
        m.tile_rows == c->tile_rows && m.spp == c->fp.spp_side && m.ntiles == ntiles) {
      m.tick = ++c->bal_clock;
      return &m;
    }
    if (!lru || m.tick < lru->tick) lru = &m;
  }
  BalanceMap* m = nullptr;
  bool recycled = false;
  c->bal.reserve(rt_ctx::kMaxBalanceMaps);  // the maps never move (bal_last points at one)
  if (c->bal.size() < rt_ctx::kMaxBalanceMaps) {
    c->bal.emplace_back();
    m = &c->bal.back();
  } else if (!forced) {
    // more live shapes than maps (e.g. 40 emulated loopback ranks, each its own row list) would recycle
    // maps in a cycle where none survives to its first plan, paying a memset and host queries per launch for a
    // balance that never runs. A map used within the last 2 x kMaxBalanceMaps lookups is not taken, and after a
    // miss the table is scanned again only every kRecycleBackoff launches of unknown shapes.
    if (c->bal_backoff) {
      --c->bal_backoff;
      ++c->bal_full;
      return nullptr;
    }
    for (BalanceMap& o : c->bal)  // the least recently used idle map that fits
      if (o.cost_cap >= ntiles && c->bal_clock - o.tick > 2 * rt_ctx::kMaxBalanceMaps && (!m || o.tick < m->tick) &&
          balance_idle(o))
        m = &o;
    if (!m) {
      ++c->bal_full;
      c->bal_backoff = rt_ctx::kRecycleBackoff;
      return nullptr;
    }
    ++c->bal_recycled;
    recycled = true;
  } else {
    // tests: the least recently used shape's buffers may still be read by launches in flight
    if ((*err = quiesce(c)) != hipSuccess) return nullptr;
    m = lru;
    if (c->bal_last == m) c->bal_last = nullptr;
    m->release();
  }
  if (recycled) {
    // keep the buffers (cost, lists, stats, events); restart the shape's state
    m->launches = 0;
    m->last_stream = nullptr;
    m->active_run = m->idle_queries = 0;
    m->cur = m->pending = -1;
    m->cur_items = m->pending_items = 0;
    m->planned_at = 0;
    m->readers.clear();
    m->streams.clear();
    m->recycled = true;
    m->recycled_planned = false;
    m->nopay_run = 0;
  }
  m->W = W;
  m->nrows = nrows;
  m->rows = d_rows;
  m->rows_gen = rows_gen;
  m->nframes = nframes;
  m->tile_rows = c->tile_rows;
  m->spp = c->fp.spp_side;
  m->ntiles = ntiles;
  // the extra waves a list may add for split tiles: an eighth of the tiles. The plan raises its threshold until the
  // parts fit, so only the heaviest tiles split (a quarter or a sixteenth measured 3-9 % slower on C4 / C2F frames
  // and shares, profiles/r04_balance_budget_sweep2.txt). (A budget that followed the plan's demand let later plans split
  // every tile above max(L, 0.35 x the costliest): rank 0's C4 share of 4 went from 120 to 167 us per launch,
  // profiles/r04_share_trace_C4_n4.txt.)
  m->extra_cap = ntiles / c->bal_budget + 64u;
  m->tick = ++c->bal_clock;
  if (recycled) {
    if ((*err = hipMemsetAsync(m->cost, 0, (size_t)ntiles * 8, s)) != hipSuccess) return nullptr;
    std::memset(m->stats, 0, sizeof(rt::PlanStats));
    return m;
  }
  m->cost_cap = ntiles;
  if ((*err = hipMalloc(&m->cost, (size_t)ntiles * 8)) != hipSuccess ||
      (*err = hipMemsetAsync(m->cost, 0, (size_t)ntiles * 8, s)) != hipSuccess ||
      (*err = hipHostMalloc((void**)&m->stats, sizeof(rt::PlanStats), hipHostMallocMapped)) != hipSuccess) {
    m->release();
    return nullptr;
  }
  std::memset(m->stats, 0, sizeof(rt::PlanStats));
  if ((*err = hipHostGetDevicePointer((void**)&m->stats_dev, m->stats, 0)) != hipSuccess) {
    m->release();
    return nullptr;
  }
  return m;
}

// Adaptive mode: whether this launch starts a plan (the next list, on the plan stream), and whether it runs with the
// shape's current list at all. Not before the shape has wave times. A list that differs from the plain order (the
// last plan's `pays`) is used by every launch and re-planned every kReplan launches (the costs drift with the
// camera); otherwise the launches take the plain grid and one in kRecheck plans again. One plan at a time per
// shape. The summary is read from host-mapped memory without a copy call (it may lag: any list is a valid cover).
constexpr uint64_t kReplan = 8, kRecheck = 32, kRecheckNoTail = 128;
// a shape whose plans keep finding nothing to gain (C2: 17 plans, none paid, in one bench run) doubles
// its re-check interval after each such plan, up to 2^kNoPayBackoff times the base (128 -> 4096 launches for C2);
// one plan that pays resets it
constexpr uint32_t kNoPayBackoff = 5;

// record: whether the launch's waves record their times. A shape whose list does not pay runs the plain kernel
// and records only on the launch before a re-check (the plan reads those times).
// A plan starts only on the second active launch in a row (the first launch after the caller drained its streams
// is active too, and a plan started there would run beside the frames in flight that follow). A shape whose last
// plan found no tail at all, or whose tiles are coherent (no split helped), re-checks every kRecheckNoTail launches,
// one whose tail splitting could not shorten every kRecheck.
static void balance_wants_plan(BalanceMap& m, bool* plan, bool* use, bool* record) {
  const volatile rt::PlanStats* st = m.stats;
  *plan = *use = false;
  *record = true;
  if (m.launches == 0) return;
  const bool may_plan = m.pending < 0 && m.active_run >= 2u;
  if (m.cur < 0) {  // the first list: the plain grid until it is ready, recording until its plan starts
    *plan = may_plan;
    *record = m.pending < 0;
    return;
  }
  const uint64_t age = m.launches - m.planned_at;
  *use = st->pays != 0;
  const uint64_t base = (st->threshold == 0xffffffffu || st->coherent) ? kRecheckNoTail : kRecheck;
  const uint32_t back = m.nopay_run > 1u ? std::min(m.nopay_run - 1u, kNoPayBackoff) : 0u;
  const uint64_t every = *use ? kReplan : base << back;
  *plan = may_plan && age >= every;
  // a launch with a list runs the recording kernel anyway; otherwise only the launch before a re-check records
  // (not every launch issued while a plan is pending: a host running far ahead issues many of those)
  *record = *use || age + 1u >= every;
}

// The current list stops being current: one event per stream that launched with it (covering all of that stream's
// launches so far), so the plan that overwrites it later orders after them on the device. On a failed record
// (a stream destroyed without rt_forget_stream) the device is drained instead.
static hipError_t balance_swap_out(BalanceMap& m) {
  hipError_t first = hipSuccess;
  if (m.cur >= 0)
    for (hipStream_t r : m.readers) {
      const hipError_t e = slot_mark_use(m.list[m.cur], r);
      if (e != hipSuccess && first == hipSuccess) first = e;
    }
  m.readers.clear();
  if (first != hipSuccess) (void)hipDeviceSynchronize();
  return first;
}

// RayGen's per-frame constants from a camera buffer (UpdateCameraBuffer's 256 B, D3D12HelloTriangle.cpp:1144-1170):
// viewInverse and projectionInverse as the HLSL reads them, and the origin mul(viewInverse, (0, 0, 0, 1)) by the
// device's own hlsl_mul4 (RT_HD, no contraction), so the kernel gets the bits it would compute.
void frame_cam(const float cb[64], FrameCam& cam) {
  std::memcpy(cam.view_inv, cb + 32, 16 * sizeof(float));
  std::memcpy(cam.proj_inv, cb + 48, 16 * sizeof(float));
  const float zero_one[4] = {0.0f, 0.0f, 0.0f, 1.0f};
  rt::hlsl_mul4(cb + 32, zero_one, cam.origin);
}

// The frame launch behind rt_dispatch_rays and rt_render_strips (d_rows: a device row list or null; the
// caller validated the arguments with check_dispatch and keeps d_rows alive until the launch completed).
// nframes frames in one launch (the grid's z): frame z with camera buffer cams[64 z ..] (null: the context's
// camera for every frame) into out + z * frame_stride bytes (0: nrows * W * out_bpp, compact); out_bpp 4 = RGBA8,
// 3 = RGB8 (strips).
rt_status dispatch_frame(rt_ctx* c, uint32_t W, uint32_t H, const uint32_t* d_rows, uint32_t nrows, void* rgba8,
                         float* rgba32f, hipStream_t s, uint32_t out_bpp, uint32_t nframes, const float* cams,
                         uint64_t frame_stride, uint64_t rows_gen) {
  if (nframes < 1 || nframes > (uint32_t)rt::kMaxLaunchFrames || (out_bpp != 3 && out_bpp != 4) ||
      (nframes > 1 && rgba32f))
    return fail(c, RT_E_INVALID, "dispatch: 1..4 frames per launch, RGBA8 or RGB8, float output for one frame only");
  const uint64_t frame_bytes = frame_stride ? frame_stride : (uint64_t)nrows * W * out_bpp;
  if (frame_bytes * nframes >= 0xffffffffull) return fail(c, RT_E_UNSUPPORTED, "dispatch: frame exceeds 4 GB");
  c->fp.width = W;
  c->fp.height = H;
  c->fp.fwidth = (float)W;  // exact: W, H < 2^24
  c->fp.fheight = (float)H;
  c->fp.nrows = nrows;
  c->fp.tile_rows = c->tile_rows;
  c->fp.out_bpp = out_bpp;
  c->fp.nframes = nframes;
  c->fp.frame_bytes = (uint32_t)frame_bytes;
  for (uint32_t z = 0; z < nframes; ++z) frame_cam(cams ? cams + 64 * z : c->cam_cb, c->fp.cam[z]);
  rt::SceneView sv = scene_view(c);
  if (sv.stack_cap > rt::kMaxTraversalStack)
    return fail(c, RT_E_UNSUPPORTED, "rt_dispatch_rays: BVH too deep for the traversal stack");
  ScratchSlot* ovf_slot = nullptr;
  {
    const size_t lanes = (size_t)((W + 15) / 16) * ((nrows + 15) / 16) * 256 * nframes;
    rt_status st = ensure_overflow(c, sv, lanes, s, &ovf_slot);
    if (st != RT_OK) return st;
  }
  HIPCHK(c, order_after_tlas(c, s), "rt_dispatch_rays: order after the TLAS build");
  // tile balance (packet schedule): the per-tile wave times of this shape, and a work list when it pays
  const rt::PacketGeometry g = rt::packet_geometry(sv, c->fp, c->schedule);
  c->fp.plan = nullptr;
  c->fp.cost = nullptr;
  c->fp.grid_x = g.grid_x;
  c->fp.waves_per_frame = g.waves_per_frame;
  uint32_t plan_items = 0;
  ScratchSlot* plan_slot = nullptr;
  const bool forced = c->balance >= 2;
  if (forced && (uint64_t)g.waves_per_frame * nframes > rt::kPlanMaxTiles)
    return fail(c, RT_E_UNSUPPORTED, "tile balance: forced layouts take at most 32768 waves per launch");
  // launches of more waves than the plan kernel holds run the plain grid (they are many rounds of the GPU's wave
  // slots deep: the slowest tile is a small part of them, C5's 518,400 waves)
  if (c->balance && g.packet && g.plannable && (forced || !c->stats_on) &&
      (uint64_t)g.waves_per_frame * nframes <= rt::kPlanMaxTiles) {
    const uint32_t ntiles = g.waves_per_frame * nframes;
    hipError_t be;
    BalanceMap* m = balance_map(c, W, nrows, d_rows, rows_gen, nframes, ntiles, s, forced, &be);
    if (!m && be != hipSuccess) return hip_fail(c, be, "tile balance: cost map");
    if (m) {
      c->bal_last = m;
      // frames in flight (the shape's previous launch still runs on another stream): the next frame's waves already
      // fill the slots the slowest tiles leave idle, so the balance only adds work there (split parts, the plan). It
      // runs when this launch follows the previous one on its stream or that stream has drained (frame latency: one
      // frame at a time, a rank's share of a frame). A host query of the stream: no event in the launch's stream.
      // While the shape is in flight the stream is queried on one launch in 16 only: frames in flight are issued as
      // fast as the host can (C1's 9-us frames are bound by the host's issue), and the query is a runtime call.
      bool active = forced || s == m->last_stream || !m->last_stream;
      if (!active && (m->active_run > 0u || (++m->idle_queries & 15u) == 0u))
        active = hipStreamQuery(m->last_stream) == hipSuccess;
      m->last_stream = s;
      m->active_run = active ? m->active_run + 1u : 0u;
      bool plan = forced, use = forced, record = false;
      // a pending list that is ready becomes the current one (the old one's readers recorded for the next plan)
      if (active && !forced && m->pending >= 0 && hipEventQuery(m->pend_ev) == hipSuccess) {
        HIPCHK(c, balance_swap_out(*m), "tile balance: record the list's readers");
        m->cur = m->pending;
        m->cur_items = m->pending_items;
        m->pending = -1;
        // the plan just landed (its event completed: its host-mapped summary is visible)
        const volatile rt::PlanStats* ps = m->stats;
        m->nopay_run = ps->pays ? 0u : m->nopay_run + 1u;
      }
      if (active && !forced) balance_wants_plan(*m, &plan, &use, &record);
      if (c->bal_diag == 1) {
        plan = use = false;
        record = true;
      } else if (c->bal_diag == 2 && (m->cur >= 0 || m->pending >= 0)) {
        record = false;
      } else if (c->bal_diag == 3 && m->cur >= 0) {
        use = true;  // the current list even where it does not pay (with RT_BALANCE_SPLIT=0 RT_BALANCE_FRONT=0: the plain order)
      }
      c->fp.cost = record ? m->cost : nullptr;
      rt::PlanArgs a;
      a.cost = m->cost;
      a.stats = forced ? nullptr : m->stats_dev;
      a.ntiles = ntiles;
      a.slots = 0;  // set below for a plan: the list's kernel's occupancy x CUs, from the runtime
      // adaptive plans split into at most 16 parts unless RT_BALANCE_FINE allows the 64 single-pixel parts
      a.kmax_code = forced ? g.kmax_code : std::min<uint32_t>(g.kmax_code, c->bal_fine ? 3u : 2u);
      a.force = forced ? (uint32_t)(c->balance - 1) : 0u;
      a.split = c->bal_split;
      a.front = c->bal_front;
      a.prio = c->bal_prio;
      a.check = c->bal_check;
      a.min_gain = 1000u;  // 10 us: above the plan kernel's own time
      a.waves_per_frame = g.waves_per_frame;
      a.grid_x = g.grid_x;
      a.wx = g.wx;
      a.wy = g.wy;
      a.wl = g.wl;
      if (forced) {
        // tests: a fresh list per launch from the ring (RT_BALANCE_FORCED_CAP, tests: a smaller budget of extra waves,
        // so the plan must refuse parts and fall back to the plain grid's list)
        // the layout's own parts (modes 2 / 3 / 4 / 5: at most 4 / 16 / 16 / 64 per tile)
      const uint32_t most = c->balance == 2 ? 4u : c->balance == 5 ? 64u : 16u;
      a.extra_cap = c->bal_forced_cap ? c->bal_forced_cap : (most - 1u) * ntiles;
        a.stats = m->stats_dev;
        a.slots = plan_slots(c, sv);
        plan_items = ntiles + a.extra_cap;
        bool hit;
        plan_slot = ring_acquire(c->plans, s, nullptr, &hit, &be);
        if (be != hipSuccess) return hip_fail(c, be, "tile balance: order after in-flight launches");
        HIPCHK(c, slot_reserve(*plan_slot, ((size_t)rt::plan_xwords(plan_items, a.wl) + 3u * ntiles + 1) * 4),
               "hipMalloc(tile plan)");
        a.plan = (uint32_t*)plan_slot->buf;
        HIPCHK(c, rt::launch_tile_plan(a, s), "tile plan launch");
        c->fp.plan = a.plan;
      } else if (active) {
        if (plan) {
          // the next list goes into the other buffer, on the plan stream, after every launch that read that buffer
          // and after this stream's earlier work (the costs it recorded); this launch keeps the current list
          hipStream_t ps = c->stream;
          const int b = m->cur < 0 ? 0 : 1 - m->cur;
          ScratchSlot& sl = m->list[b];
          if ((!m->pend_ev && !(m->pend_ev = new_sync_event())) || (!m->src_ev && !(m->src_ev = new_sync_event())))
            return fail(c, RT_E_HIP, "tile balance: event");
          HIPCHK(c, hipEventRecord(m->src_ev, s), "tile balance: record the launch stream");
          HIPCHK(c, hipStreamWaitEvent(ps, m->src_ev, 0), "tile balance: order the plan");
          HIPCHK(c, slot_order_after_others(sl, ps), "tile balance: order after the list's readers");
          a.extra_cap = m->extra_cap;
          a.slots = plan_slots(c, sv);
          const uint32_t items = ntiles + a.extra_cap;
          HIPCHK(c, slot_reserve(sl, ((size_t)rt::plan_xwords(items, a.wl) + 3u * ntiles + 1) * 4), "hipMalloc(tile plan)");
          a.plan = (uint32_t*)sl.buf;
          HIPCHK(c, rt::launch_tile_plan(a, ps), "tile plan launch");
          HIPCHK(c, hipEventRecord(m->pend_ev, ps), "tile balance: record the plan");
          m->pending = b;
          m->pending_items = items;
          m->planned_at = m->launches;
          if (m->recycled && !m->recycled_planned) {
            m->recycled_planned = true;
            ++c->bal_recycled_planned;
          }
        }
        if (use && m->cur >= 0) {
          if (std::find(m->readers.begin(), m->readers.end(), s) == m->readers.end()) m->readers.push_back(s);
          c->fp.plan = (const uint32_t*)m->list[m->cur].buf;
          plan_items = m->cur_items;
        }
      }
      if (active) m->launches += 1;
      // the streams whose launches read or write the map's buffers (its recycling waits until all are idle)
      if ((c->fp.cost || c->fp.plan) && std::find(m->streams.begin(), m->streams.end(), s) == m->streams.end())
        m->streams.push_back(s);
    }
  }
  hipError_t e = rt::launch_trace_frame(sv, c->fp, d_rows, rgba8, rgba32f, c->d_stats, c->stats_on,
                                        c->schedule, plan_items, s);
  if (e != hipSuccess) return hip_fail(c, e, "trace launch");
  HIPCHK(c, note_reader(c->ver[c->cur], s), "rt_dispatch_rays: record use");
  if (ovf_slot) HIPCHK(c, slot_mark_use(*ovf_slot, s), "overflow stack: record use");
  if (plan_slot) HIPCHK(c, slot_mark_use(*plan_slot, s), "tile plan: record use");
  if (c->stats_on) {
    c->dispatches += nframes;
    c->pixels += (uint64_t)W * nrows * nframes;
  }
  return RT_OK;
}

}  // namespace rt

extern "C" {

rt_status rt_raster_draw(rt_ctx_t c, const rt_blas_t* draws, uint32_t ndraws, const float* object_to_world,
                         uint32_t W, uint32_t H, void* rgba8, float* depth32f, void* stream) {
  if (!c) return RT_E_INVALID;
  if (!draws || ndraws == 0 || ndraws > rt::kRasterMaxDraws)
    return fail(c, RT_E_INVALID, "rt_raster_draw: 1..8 draws required");
  if (!c->have_camera) return fail(c, RT_E_INVALID, "rt_raster_draw: camera not set");
  if (W == 0 || H == 0 || W > 16384 || H > 16384 || !rgba8)
    return fail(c, RT_E_INVALID, "rt_raster_draw: bad size or output");
  rt::RasterDraws dr;
  dr.n = ndraws;
  uint64_t total = 0;
  for (uint32_t d = 0; d < ndraws; ++d) {
    if (draws[d] >= c->blas.size() || !c->blas[draws[d]].vtx) return fail(c, RT_E_INVALID, "rt_raster_draw: unknown BLAS");
    const DeviceBlas& b = c->blas[draws[d]];
    dr.first[d] = (uint32_t)total;
    dr.nvtx[d] = b.nvtx;
    dr.vtx[d] = b.vtx;
    dr.idx[d] = b.idx;
    total += b.ntri;
  }
  if (total * 7 >= 0xffffffffull) return fail(c, RT_E_UNSUPPORTED, "rt_raster_draw: too many triangles");
  dr.total = (uint32_t)total;
  rt::RasterView rv;
  // objectToWorld as the instance properties buffer holds it (XMMATRIX memory, row-vector
  // convention): memory row j = column j of the 3x4 column-vector transform
  const float I[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
  const float* T = object_to_world ? object_to_world : I;
  for (int j = 0; j < 4; ++j) {
    for (int i = 0; i < 3; ++i) rv.o2w[j * 4 + i] = T[i * 4 + j];
    rv.o2w[j * 4 + 3] = j == 3 ? 1.0f : 0.0f;
  }
  std::memcpy(rv.view, c->cam_cb, 16 * sizeof(float));
  std::memcpy(rv.proj, c->cam_cb + 16, 16 * sizeof(float));
  rv.width = W;
  rv.height = H;
  (void)hipSetDevice(c->device);
  hipStream_t s = pick_stream(c, stream);
  const size_t ntiles = (size_t)((W + 7) / 8) * ((H + 7) / 8);
  auto regrow = [&](void** p, size_t bytes, const char* what) -> rt_status {
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    HIPCHK(c, hipMalloc(p, bytes), what);
    return RT_OK;
  };
  rt_status st = RT_OK;
  if (c->raster_tile_cap < ntiles || c->raster_prim_cap < total) {
    HIPCHK(c, quiesce(c), "rt_raster_draw: wait for in-flight work");
    if (c->raster_tile_cap < ntiles) {
      if ((st = regrow((void**)&c->raster.tcount, ntiles * 4, "hipMalloc(raster tile counts)")) != RT_OK) return st;
      if ((st = regrow((void**)&c->raster.toffs, (ntiles + 1) * 4, "hipMalloc(raster tile offsets)")) != RT_OK) return st;
      if ((st = regrow((void**)&c->raster.bsum, (ntiles / 4096 + 2) * 4, "hipMalloc(raster scan)")) != RT_OK) return st;
      if (!c->raster.draws &&
          (st = regrow((void**)&c->raster.draws, sizeof(rt::RasterDraws), "hipMalloc(raster draws)")) != RT_OK)
        return st;
      c->raster_tile_cap = ntiles;
    }
    if (c->raster_prim_cap < total) {
      const size_t n = (size_t)total;
      if ((st = regrow((void**)&c->raster.clip, n * 3 * sizeof(float4), "hipMalloc(raster clip)")) != RT_OK) return st;
      if ((st = regrow((void**)&c->raster.slots, n * 7 * sizeof(rt::RasterSlot), "hipMalloc(raster slots)")) != RT_OK)
        return st;
      if ((st = regrow((void**)&c->raster.tiles, n * 7 * 4, "hipMalloc(raster slot tiles)")) != RT_OK) return st;
      c->raster_prim_cap = n;
    }
  }
  if (!c->raster_total_host) {
    HIPCHK(c, hipHostMalloc((void**)&c->raster_total_host, 4, hipHostMallocDefault), "hipHostMalloc(raster total)");
    *c->raster_total_host = 0;
  }
  // the draw list on the device changes only with the draws (or a BLAS rebuild): uploaded then,
  // not per draw, so nothing of a draw reads host memory after the call returns
  if (std::memcmp(&c->raster_draws_host, &dr, sizeof(dr)) != 0) {
    HIPCHK(c, quiesce(c), "rt_raster_draw: wait for in-flight work");
    HIPCHK(c, hipMemcpy(c->raster.draws, &dr, sizeof(dr), hipMemcpyHostToDevice), "upload raster draws");
    c->raster_draws_host = dr;
  }
  // bins are sized from a bin-entry total already known on the host: the first draw reads its own
  // (one synchronisation), later draws the last total copied back asynchronously. A draw with more
  // entries than that capacity still renders the same image (k_raster_tile walks every slot) and
  // the next draw grows the bins.
  const uint32_t last_total = *(volatile uint32_t*)c->raster_total_host;
  // one raster scratch per context: a draw on another stream than the previous draw's runs after it
  if (c->raster_pending && c->raster_stream != s) {
    if (hipEventQuery(c->raster_ev) == hipSuccess) c->raster_pending = false;
    else HIPCHK(c, hipStreamWaitEvent(s, c->raster_ev, 0), "rt_raster_draw: order after the previous draw");
  }
  hipError_t e = rt::launch_raster_bin(dr, rv, c->raster, s);
  if (e != hipSuccess) return hip_fail(c, e, "raster bin launch");
  size_t want = 0;
  if (c->raster_bin_cap == 0) {
    uint32_t nbins = 0;
    HIPCHK(c, hipMemcpyAsync(&nbins, c->raster.toffs + ntiles, 4, hipMemcpyDeviceToHost, s), "raster bin count");
    HIPCHK(c, hipStreamSynchronize(s), "raster bin count");
    want = (size_t)nbins + nbins / 2 + 64;
  } else if (last_total > c->raster_bin_cap) {
    want = (size_t)last_total + last_total / 2;
  }
  // test hook: RT_RASTER_BIN_CAP caps the capacity (forces the slot-walk path)
  if (const char* ev = std::getenv("RT_RASTER_BIN_CAP")) {
    const size_t lim = (size_t)std::strtoull(ev, nullptr, 10);
    if (want == 0 && c->raster_bin_cap > lim) want = lim;
    if (want > lim) want = lim;
  }
  if (want != 0 && want != c->raster_bin_cap) {
    HIPCHK(c, quiesce(c), "rt_raster_draw: wait for in-flight work");
    if ((st = regrow((void**)&c->raster.bins, (want ? want : 1) * 4, "hipMalloc(raster bins)")) != RT_OK) return st;
    c->raster_bin_cap = want;
  }
  const uint32_t cap = (uint32_t)std::min<size_t>(c->raster_bin_cap, 0xffffffffu);
  e = rt::launch_raster_draw(dr, rv, c->raster, cap, rgba8, depth32f, s);
  if (e != hipSuccess) return hip_fail(c, e, "raster launch");
  HIPCHK(c, hipMemcpyAsync(c->raster_total_host, c->raster.toffs + ntiles, 4, hipMemcpyDeviceToHost, s),
         "raster bin total");
  if (!c->raster_ev && !(c->raster_ev = new_sync_event())) return fail(c, RT_E_HIP, "rt_raster_draw: event");
  HIPCHK(c, hipEventRecord(c->raster_ev, s), "rt_raster_draw: record");
  c->raster_stream = s;
  c->raster_pending = true;
  return RT_OK;
}

rt_status rt_dispatch_rays(rt_ctx_t c, uint32_t W, uint32_t H, const uint32_t* rows, uint32_t nrows,
                           void* rgba8, float* rgba32f, void* stream) {
  if (!c) return RT_E_INVALID;
  if (!rows) nrows = H;
  if (nrows == 0 || nrows > H) return fail(c, RT_E_INVALID, "rt_dispatch_rays: bad row count");
  if (rows)
    for (uint32_t r = 0; r < nrows; ++r)
      if (rows[r] >= H) return fail(c, RT_E_INVALID, "rt_dispatch_rays: row index out of range");
  (void)hipSetDevice(c->device);
  hipStream_t s = pick_stream(c, stream);
  rt_status st = rt::check_dispatch(c, W, H, rgba8);
  if (st != RT_OK) return st;
  const uint32_t* d_rows = nullptr;
  ScratchSlot* rows_slot = nullptr;
  uint64_t rows_gen = 0;
  if (rows && (st = ensure_rows(c, rows, nrows, s, &rows_slot, &d_rows, &rows_gen)) != RT_OK) return st;
  if ((st = rt::dispatch_frame(c, W, H, d_rows, nrows, rgba8, rgba32f, s, 4, 1, nullptr, 0, rows_gen)) != RT_OK)
    return st;
  if (rows_slot) HIPCHK(c, slot_mark_use(*rows_slot, s), "rows: record use");
  return RT_OK;
}

rt_status rt_dispatch_frames(rt_ctx_t c, uint32_t W, uint32_t H, uint32_t nframes, const float* cameras,
                             void* rgba8, uint64_t frame_stride, void* stream) {
  if (!c) return RT_E_INVALID;
  if (nframes < 1 || nframes > (uint32_t)rt::kMaxLaunchFrames)
    return fail(c, RT_E_INVALID, "rt_dispatch_frames: 1..4 frames per launch");
  if (frame_stride && frame_stride < (uint64_t)W * H * 4)
    return fail(c, RT_E_INVALID, "rt_dispatch_frames: frame stride below one frame");
  if (frame_stride % 4)  // the RGBA8 stores are 32-bit words
    return fail(c, RT_E_INVALID, "rt_dispatch_frames: frame stride not a multiple of 4 bytes");
  (void)hipSetDevice(c->device);
  hipStream_t s = pick_stream(c, stream);
  rt_status st = rt::check_dispatch(c, W, H, rgba8, cameras != nullptr);
  if (st != RT_OK) return st;
  return rt::dispatch_frame(c, W, H, nullptr, H, rgba8, nullptr, s, 4, nframes, cameras, frame_stride, 0);
}

rt_status rt_trace_rays(rt_ctx_t c, const float* rays, uint32_t n, uint32_t ray_flags, uint32_t* hits, float* uv,
                        void* stream) {
  if (!c || (!rays && n) || (!hits && n)) return fail(c, RT_E_INVALID, "rt_trace_rays: null argument");
  if (ray_flags & ~(uint32_t)(RT_RAY_FLAG_ACCEPT_FIRST_HIT_AND_END_SEARCH | RT_RAY_FLAG_CULL_BACK_FACING_TRIANGLES |
                              RT_RAY_FLAG_CULL_FRONT_FACING_TRIANGLES))
    return fail(c, RT_E_INVALID, "rt_trace_rays: unsupported ray flags");
  const bool cull_back = (ray_flags & RT_RAY_FLAG_CULL_BACK_FACING_TRIANGLES) != 0;
  const bool cull_front = (ray_flags & RT_RAY_FLAG_CULL_FRONT_FACING_TRIANGLES) != 0;
  if (cull_back && cull_front) return fail(c, RT_E_INVALID, "rt_trace_rays: both cull flags set");
  if (c->cur < 0 && !c->tlas_stale) return fail(c, RT_E_INVALID, "rt_trace_rays: no TLAS built");
  if (c->tlas_stale)
    return fail(c, RT_E_INVALID, "rt_trace_rays: scene stale (BLAS rebuilt, or the last rt_tlas_build failed)");
  (void)hipSetDevice(c->device);
  rt::SceneView sv = scene_view(c);
  sv.cull_sense = cull_front ? -1.0f : 1.0f;
  if (sv.stack_cap > rt::kMaxTraversalStack)
    return fail(c, RT_E_UNSUPPORTED, "rt_trace_rays: BVH too deep for the traversal stack");
  if (n == 0) return RT_OK;
  hipStream_t s = pick_stream(c, stream);
  ScratchSlot* ovf_slot = nullptr;
  {
    rt_status st = ensure_overflow(c, sv, (size_t)((n + 255) / 256) * 256, s, &ovf_slot);
    if (st != RT_OK) return st;
  }
  HIPCHK(c, order_after_tlas(c, s), "rt_trace_rays: order after the TLAS build");
  hipError_t e = rt::launch_trace_rays(sv, rays, n, (ray_flags & RT_RAY_FLAG_ACCEPT_FIRST_HIT_AND_END_SEARCH) != 0,
                                       cull_back || cull_front, hits, uv, c->d_stats, c->stats_on, s);
  if (e != hipSuccess) return hip_fail(c, e, "trace_rays launch");
  HIPCHK(c, note_reader(c->ver[c->cur], s), "rt_trace_rays: record use");
  if (ovf_slot) HIPCHK(c, slot_mark_use(*ovf_slot, s), "overflow stack: record use");
  return RT_OK;
}

rt_status rt_assemble_strips(rt_ctx_t c, uint32_t W, uint32_t H, uint32_t nranks, uint32_t strip_rows,
                             const void* gathered, void* out, void* stream) {
  if (!c || !gathered || !out || W == 0 || H == 0 || nranks == 0 || strip_rows == 0)
    return fail(c, RT_E_INVALID, "rt_assemble_strips: bad argument");
  (void)hipSetDevice(c->device);
  hipError_t e = rt::launch_assemble_strips(W, H, nranks, strip_rows, gathered, out, pick_stream(c, stream));
  if (e != hipSuccess) return hip_fail(c, e, "assemble launch");
  return RT_OK;
}

uint32_t rt_strip_rows(uint32_t H, uint32_t nranks, uint32_t rank, uint32_t strip_rows, uint32_t* rows_out,
                       uint32_t cap) {
  if (nranks == 0 || rank >= nranks || strip_rows == 0) return 0;
  uint32_t n = 0;
  const uint32_t nstrips = (H + strip_rows - 1) / strip_rows;
  for (uint32_t s = rank; s < nstrips; s += nranks)
    for (uint32_t r = s * strip_rows; r < H && r < (s + 1) * strip_rows; ++r) {
      if (rows_out && n < cap) rows_out[n] = r;
      ++n;
    }
  return n;
}

rt_status rt_forget_stream(rt_ctx_t c, void* stream) {
  if (!c || !stream) return RT_E_INVALID;
  (void)hipSetDevice(c->device);
  HIPCHK(c, rt::ctx_forget_stream(c, (hipStream_t)stream), "rt_forget_stream");
  return RT_OK;
}

rt_status rt_event_create(void** ev_out) {
  if (!ev_out) return RT_E_INVALID;
  *ev_out = nullptr;
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess) return RT_E_HIP;
  *ev_out = e;
  return RT_OK;
}

rt_status rt_event_destroy(void* ev) {
  if (!ev) return RT_E_INVALID;
  return hipEventDestroy((hipEvent_t)ev) == hipSuccess ? RT_OK : RT_E_HIP;
}

rt_status rt_event_record(void* ev, void* stream) {
  if (!ev) return RT_E_INVALID;
  return hipEventRecord((hipEvent_t)ev, (hipStream_t)stream) == hipSuccess ? RT_OK : RT_E_HIP;
}

rt_status rt_stream_wait_event(void* stream, void* ev) {
  if (!ev) return RT_E_INVALID;
  return hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)ev, 0) == hipSuccess ? RT_OK : RT_E_HIP;
}

rt_status rt_stats(rt_ctx_t c, uint64_t out[RT_STAT_COUNT]) {
  if (!c || !out) return RT_E_INVALID;
  (void)hipSetDevice(c->device);
  HIPCHK(c, hipDeviceSynchronize(), "stats sync");
  unsigned long long h[RT_STAT_COUNT];
  HIPCHK(c, hipMemcpy(h, c->d_stats, sizeof(h), hipMemcpyDeviceToHost), "stats copy");
  for (int k = 0; k < 6; ++k) out[k] = h[k];
  out[RT_STAT_PIXELS] = c->pixels;
  out[RT_STAT_DISPATCHES] = c->dispatches;
  for (int k = RT_STAT_REFLECTION_RAYS; k < RT_STAT_COUNT; ++k) out[k] = h[k];
  return RT_OK;
}

rt_status rt_stats_reset(rt_ctx_t c) {
  if (!c) return RT_E_INVALID;
  (void)hipSetDevice(c->device);
  // hipMemset runs on the null stream, which the context's non-blocking stream does not wait for: drain the
  // device, clear, and drain again, so no counting launch before or after can straddle the reset
  HIPCHK(c, hipDeviceSynchronize(), "stats reset");
  HIPCHK(c, hipMemset(c->d_stats, 0, RT_STAT_COUNT * sizeof(unsigned long long)), "stats reset");
  HIPCHK(c, hipDeviceSynchronize(), "stats reset");
  c->pixels = 0;
  c->dispatches = 0;
  return RT_OK;
}

}  // extern "C"
