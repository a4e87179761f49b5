// rt_comm.cpp — the multi-GPU frame loop behind the C-ABI: one frame tiled over the
// ranks in interleaved strips, ONE ncclGather of every rank's compact strip buffer into rank 0
// (rccl.h:745), then the un-interleave kernel (rt_assemble_strips) on rank 0. One process per GPU,
// each with its own rt_ctx and the full scene; nothing but finished strips crosses xGMI.
//
// The frame being tiled is the reference's DispatchRays W x H (D3D12HelloTriangle.cpp:584-592),
// issued once per OnRender (:436-471). The whole step is issued from C++, so a step costs one call of
// host issue instead of a Python loop of collectives.
//
// Two host threads issue a step. The caller's thread renders the slot on its render stream and records the
// render event; the communicator's issue thread orders the gather after it (one device-side wait), issues the
// ncclGather on the gather stream and records its completion. The step's tail goes back to the slot's render
// stream, issued by the caller's thread: a wait for that gather, then rank 0's assembly. The caller issues a tail
// at a later call once the issue thread has enqueued its gather, so it does not wait for the issue thread, and at
// the latest before the slot renders again (or at rt_comm_stream / rt_comm_synchronize). With rt_comm_set_batch(b),
// b consecutive frames fill one slot (each at its own offset) and share ONE ncclGather and one tail. So the gather stream carries nothing but the gathers, and the
// slot's next render on its stream follows its tail in stream order (no release event). HIP and RCCL host
// calls cost microseconds each, so the calls of a step are split over the two threads. With the
// communicator's own render streams (render_stream NULL), the gather stream and the three render streams sit
// on the four hardware queues (GPU_MAX_HW_QUEUES), so no render queues behind a gather.
//
// The strips cross xGMI as RGB8 (3 bytes a pixel): the frame's alpha byte is the constant 255, restored by the
// assembly. rt_render_strips_frames renders up to rt_comm_batch frames (one camera each) in ONE launch per rank.
//
// RCCL is bound at run time (dlopen of librccl.so.1): a process that already loaded RCCL (torch)
// shares that copy, and a context that never creates a communicator never loads it. A loopback communicator
// (rt_comm_init_loopback, tests) stands in for N ranks on one GPU without RCCL: every rank's strips are rendered
// by this process into that rank's block of the slot, and the "gather" is a device copy into rank 0's rank-major
// layout on the gather stream, issued by the issue thread where ncclGather would be; plan, batching, events, tails
// and the rank-strided assembly are those of the RCCL path.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rt_api.h"
#include "rt_internal.hpp"

namespace {

struct RcclApi {
  bool ok = false;
  std::string err;
  ncclResult_t (*getUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*commInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*commAbort)(ncclComm_t) = nullptr;  // rt_comm_abort (optional: older RCCL builds may lack it)
  ncclResult_t (*gather)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  const char* (*getErrorString)(ncclResult_t) = nullptr;
};

RcclApi& rccl() {
  static RcclApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char* e = dlerror();
      api.err = std::string("dlopen(librccl.so.1): ") + (e ? e : "not found");
      return;
    }
    auto sym = [&](const char* n) { return dlsym(h, n); };
    api.getUniqueId = (decltype(api.getUniqueId))sym("ncclGetUniqueId");
    api.commInitRank = (decltype(api.commInitRank))sym("ncclCommInitRank");
    api.commDestroy = (decltype(api.commDestroy))sym("ncclCommDestroy");
    api.commAbort = (decltype(api.commAbort))sym("ncclCommAbort");
    api.gather = (decltype(api.gather))sym("ncclGather");
    api.getErrorString = (decltype(api.getErrorString))sym("ncclGetErrorString");
    api.ok = api.getUniqueId && api.commInitRank && api.commDestroy && api.gather && api.getErrorString;
    if (!api.ok) api.err = "librccl.so.1 lacks ncclGather / ncclCommInitRank";
  });
  return api;
}

// frames per gather (rt_comm_set_batch): a slot holds up to this many consecutive frames' strips
constexpr uint32_t kMaxBatch = 4;

// bytes per pixel of the strips moved by the gather: RGB8 (the alpha byte, always 255, is restored on rank 0)
constexpr uint32_t kStripBpp = 3;

struct Slot {
  void* local = nullptr;     // this rank's strips, compact: batch x rows_per_rank x W RGB8 (frame-major); loopback:
                             // one such block per emulated rank, rank r's at r x local_bytes
  void* gathered = nullptr;  // rank 0: nranks x (batch x rows_per_rank) x W RGB8 (rank-major, as ncclGather lays it)
  hipEvent_t rendered = nullptr;  // on the slot's render stream, after its render
  hipEvent_t gathered_ev = nullptr;  // on the gather stream, after its gather
  hipEvent_t moved = nullptr;     // recorded on demand (a slot moved to another stream)
  hipEvent_t fin[kMaxBatch] = {};  // on the slot's render stream after frame b's tail, for a frame issued on another
  hipStream_t last = nullptr;     // the stream of the slot's last step (caller thread)
  bool used = false;
  // the stream and frames of the slot's last assemblies, an event recorded on demand (caller thread)
  hipStream_t asm_stream = nullptr;
  void* asm_frames[kMaxBatch] = {};
  uint32_t asm_n = 0;
  hipEvent_t asm_order = nullptr;
};

// frames in the pipeline: one slot per render stream of the communicator, as many as the hardware queues
// beside the gather stream's allow (GPU_MAX_HW_QUEUES - 1: 3 at HIP's default of 4), at most kMaxSlots
constexpr uint32_t kMaxSlots = 8;

hipEvent_t pipeline_event() {
  hipEvent_t e = nullptr;
  // device-side hand-offs only: no timestamp, no system-scope release (rt_event_create's flags)
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess) return nullptr;
  return e;
}

}  // namespace

// rt_comm_set_phase_timing: one timed interval of a step on the device (a pair of timing events on one stream)
enum PhaseKind { kPhaseRender = 0, kPhaseGather = 1, kPhaseAssembly = 2, kPhases = 3 };
struct PhaseSpan {
  hipEvent_t a = nullptr, b = nullptr;
  int kind = 0;
};

struct Job {
  uint32_t slot = 0;
  uint32_t nframes = 0;              // frames in the slot (their strips are gathered by one ncclGather)
  void* frame_out[kMaxBatch] = {};   // rank 0's output frame of each
  hipStream_t fs[kMaxBatch] = {};    // the render stream a frame was issued on when it is not the slot's (or null):
                                     // its render waited for that stream, its tail is returned to it by an event
  hipStream_t rs = nullptr;          // the slot's render stream: its assembly runs there
  uint32_t W = 0, H = 0, strip = 0, rows_per_rank = 0;
  uint64_t seq = 0;
};

struct rt_comm {
  rt_ctx_t ctx = nullptr;
  int device = 0;
  uint32_t nranks = 1, rank = 0;
  bool loopback = false;  // rt_comm_init_loopback: every rank emulated by this process, no RCCL
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;  // the gathers
  // the communicator's own render streams (render_stream NULL: slot k renders on rstreams[k]), created right
  // after `stream`, so the four take four different hardware queues (HIP deals a process's streams over
  // GPU_MAX_HW_QUEUES = 4 queues in creation order): no render shares the gathers' queue
  uint32_t nslots = 3;
  hipStream_t rstreams[kMaxSlots] = {};
  hipEvent_t join[kMaxSlots] = {};  // rt_comm_stream's joins
  std::string err;
  // frame geometry of the slots (re-planned when it changes)
  uint32_t W = 0, H = 0, strip = 0, rows_per_rank = 0;
  std::vector<uint32_t> rows;  // this rank's global rows, output order (loopback: every rank's in turn)
  uint32_t* d_rows = nullptr;  // ... on the device (uploaded once per plan)
  uint64_t rows_gen = 0;       // ... its generation (rt::ctx_next_rows_gen, per plan)
  std::vector<uint32_t> lb_first, lb_count;  // loopback: rank r's rows are rows[lb_first[r] ..][0 .. lb_count[r])
  uint32_t lb_render_first = 0, lb_render_count = 0;  // rt_comm_loopback_render_ranks (0: every emulated rank)
  size_t local_bytes = 0;      // one rank's block of a slot: batch x rows_per_rank x W x kStripBpp
  hipEvent_t xev = nullptr;    // a frame issued on another stream than its slot's: the slot's stream waits for it
  // RT_COMM_TIMING=1 (diagnostics): host time per part of rt_render_strips, printed by rt_comm_destroy
  bool timing = false;
  double t_parts[6] = {0, 0, 0, 0, 0, 0};
  uint64_t t_calls = 0;
  Slot slots[kMaxSlots];
  uint64_t next = 0;  // slots started
  // frames per gather (rt_comm_set_batch, the same on every rank) and the slot being filled: its frames so far
  uint32_t batch = 1, planned_batch = 0;
  uint32_t fill = 0;
  Job cur{};
  // the issue thread of the gather side (see the header comment)
  std::thread worker;
  std::mutex mu;
  std::condition_variable cv_job, cv_done;
  std::atomic<uint64_t> posted{0};     // jobs handed over (read by the issue thread while it spins)
  std::atomic<bool> sleeping{false};   // the issue thread waits on cv_job (the caller notifies only then)
  std::deque<Job> jobs;
  uint64_t issued = 0;          // jobs handed over (caller thread)
  uint64_t done = 0;            // jobs whose gather (and its event) are enqueued (issue thread)
  uint64_t slot_seq[kMaxSlots] = {};  // the last job of each slot
  // the steps whose tail (back on its render stream: the wait for its gather, rank 0's assembly) the caller thread
  // has not issued yet, oldest first. A tail is issued at a later call once the issue thread has enqueued its
  // gather (no waiting), and at the latest before its slot renders again (waiting if the issue thread is behind)
  std::deque<Job> tails;
  bool stop = false;
  bool aborting = false;        // rt_comm_abort: the issue thread drops its queue and returns
  rt_status werr = RT_OK;       // the issue thread's first failure, returned by the next call
  std::string wmsg;
  double w_parts[3] = {0, 0, 0};  // RT_COMM_TIMING: issue-thread hand-off, ncclGather, gather event
  // rt_comm_set_phase_timing (what a step costs, per phase, on this rank): timing-event pairs around
  // the render launches (render stream), the gather (gather stream, from the moment the render is done) and rank
  // 0's assembly, resolved into sums once complete; the host time of the caller's calls and of the issue thread
  bool phase = false;  // written only with the pipeline drained; the issue thread reads it per job, after the job's
                       // hand-off under `mu` (so the write happens-before every read that can see a new job)
  std::mutex pmu;                 // the two threads record spans
  std::vector<hipEvent_t> pfree;  // resolved events, reused
  std::deque<PhaseSpan> ppend;    // recorded spans not yet resolved
  double p_ms[kPhases] = {0, 0, 0};
  uint64_t p_n[kPhases] = {0, 0, 0};
  uint64_t p_frames = 0, p_calls = 0, p_launches = 0;
  double p_host_us = 0, p_issue_us = 0;
  double p_bytes_in = 0, p_bytes = 0;  // bytes into rank 0 from the other ranks; every rank's block
};

namespace {

rt_status cfail(rt_comm* c, rt_status st, const std::string& m) {
  if (c) c->err = m;
  return st;
}

// phase timing: an event with a timestamp (no system-scope fence: the host only reads the time)
hipEvent_t phase_event(rt_comm* c) {
  {
    std::lock_guard<std::mutex> lk(c->pmu);
    if (!c->pfree.empty()) {
      hipEvent_t e = c->pfree.back();
      c->pfree.pop_back();
      return e;
    }
  }
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
  return e;
}

// records the start of a span on s (null when phase timing is off or an event could not be had)
hipEvent_t phase_begin(rt_comm* c, hipStream_t s) {
  if (!c->phase) return nullptr;
  hipEvent_t a = phase_event(c);
  if (a && hipEventRecord(a, s) != hipSuccess) {
    std::lock_guard<std::mutex> lk(c->pmu);
    c->pfree.push_back(a);
    return nullptr;
  }
  return a;
}

void phase_end(rt_comm* c, hipStream_t s, hipEvent_t a, int kind) {
  if (!a) return;
  hipEvent_t b = phase_event(c);
  std::lock_guard<std::mutex> lk(c->pmu);
  if (!b || hipEventRecord(b, s) != hipSuccess) {
    c->pfree.push_back(a);
    if (b) c->pfree.push_back(b);
    return;
  }
  PhaseSpan sp;
  sp.a = a;
  sp.b = b;
  sp.kind = kind;
  c->ppend.push_back(sp);
}

// resolves the recorded spans into the sums: those complete (wait = false), or all of them (wait = true)
void phase_collect(rt_comm* c, bool wait) {
  std::lock_guard<std::mutex> lk(c->pmu);
  std::deque<PhaseSpan> keep;
  for (const PhaseSpan& sp : c->ppend) {
    if (wait) (void)hipEventSynchronize(sp.b);
    else if (hipEventQuery(sp.b) != hipSuccess) {
      keep.push_back(sp);
      continue;
    }
    float ms = 0.0f;
    if (hipEventElapsedTime(&ms, sp.a, sp.b) == hipSuccess) {
      c->p_ms[sp.kind] += ms;
      c->p_n[sp.kind] += 1;
    }
    c->pfree.push_back(sp.a);
    c->pfree.push_back(sp.b);
  }
  c->ppend.swap(keep);
}

void phase_reset(rt_comm* c) {
  phase_collect(c, true);
  std::lock_guard<std::mutex> lk(c->pmu);
  for (int k = 0; k < kPhases; ++k) c->p_ms[k] = 0.0, c->p_n[k] = 0;
  c->p_frames = c->p_calls = c->p_launches = 0;
  c->p_host_us = c->p_issue_us = 0.0;
  c->p_bytes_in = c->p_bytes = 0.0;
}

rt_status nccl_fail(rt_comm* c, ncclResult_t r, const char* what) {
  return cfail(c, RT_E_RCCL, std::string(what) + ": " + rccl().getErrorString(r));
}

void release_slots(rt_comm* c) {
  if (c->d_rows) (void)hipFree(c->d_rows);
  c->d_rows = nullptr;
  for (Slot& s : c->slots) {
    if (s.local) (void)hipFree(s.local);
    if (s.gathered) (void)hipFree(s.gathered);
    for (hipEvent_t e : {s.rendered, s.gathered_ev, s.moved, s.asm_order})
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : s.fin)
      if (e) (void)hipEventDestroy(e);
    s = Slot();
  }
}

void wait_issued(rt_comm* c, uint64_t seq);
rt_status issue_tails(rt_comm* c, uint64_t upto);

rt_status finish_slot(rt_comm* c);

// waits (host) for every step handed over so far (a partly filled slot is handed over first): its gather on the
// gather stream, its assembly on its render stream
rt_status drain(rt_comm* c) {
  rt_status st = finish_slot(c);  // a partly filled slot is gathered as it is (every rank has filled it alike)
  if (st != RT_OK) return st;
  st = issue_tails(c, ~0ull);
  if (st != RT_OK) return st;
  wait_issued(c, c->issued);
  if (c->stream && hipStreamSynchronize(c->stream) != hipSuccess) return cfail(c, RT_E_HIP, "rt_render_strips: drain");
  for (Slot& s : c->slots)
    if (s.used && hipStreamSynchronize(s.last) != hipSuccess) return cfail(c, RT_E_HIP, "rt_render_strips: drain");
  return RT_OK;
}

// (re)plans the strips of a W x H frame and sizes the pipeline slots; waits for the slots' last uses
rt_status plan(rt_comm* c, uint32_t W, uint32_t H, uint32_t strip) {
  if (c->W == W && c->H == H && c->strip == strip && c->planned_batch == c->batch) return RT_OK;
  rt_status st = drain(c);
  if (st != RT_OK) return st;
  release_slots(c);
  c->W = c->H = c->strip = 0;
  c->rows.clear();
  c->lb_first.clear();
  c->lb_count.clear();
  // the ranks this process renders: its own, or (loopback) all of them
  const uint32_t r0 = c->loopback ? 0 : c->rank, r1 = c->loopback ? c->nranks : c->rank + 1;
  for (uint32_t r = r0; r < r1; ++r) {
    const uint32_t n = rt_strip_rows(H, c->nranks, r, strip, nullptr, 0);
    c->lb_first.push_back((uint32_t)c->rows.size());
    c->lb_count.push_back(n);
    c->rows.resize(c->rows.size() + n);
    if (n) rt_strip_rows(H, c->nranks, r, strip, c->rows.data() + c->lb_first.back(), n);
  }
  const size_t n = c->rows.size();
  if (n) {
    if (hipMalloc(&c->d_rows, n * 4) != hipSuccess) return cfail(c, RT_E_OOM, "rt_render_strips: hipMalloc(rows)");
    if (hipMemcpy(c->d_rows, c->rows.data(), n * 4, hipMemcpyHostToDevice) != hipSuccess)
      return cfail(c, RT_E_HIP, "rt_render_strips: upload rows");
  }
  c->rows_gen = rt::ctx_next_rows_gen(c->ctx);
  const uint32_t nstrips = (H + strip - 1) / strip;
  c->rows_per_rank = ((nstrips + c->nranks - 1) / c->nranks) * strip;
  c->local_bytes = (size_t)c->rows_per_rank * W * kStripBpp * c->batch;
  const size_t blocks = c->loopback ? c->nranks : 1;
  for (uint32_t k = 0; k < c->nslots; ++k) {
    Slot& s = c->slots[k];
    if (hipMalloc(&s.local, c->local_bytes * blocks) != hipSuccess)
      return cfail(c, RT_E_OOM, "rt_render_strips: hipMalloc(local)");
    if (c->rank == 0 && hipMalloc(&s.gathered, c->local_bytes * c->nranks) != hipSuccess)
      return cfail(c, RT_E_OOM, "rt_render_strips: hipMalloc(gathered)");
    if (!(s.rendered = pipeline_event()) || !(s.gathered_ev = pipeline_event()) || !(s.moved = pipeline_event()) ||
        !(s.asm_order = pipeline_event()))
      return cfail(c, RT_E_HIP, "rt_render_strips: events");
    for (hipEvent_t& e : s.fin)
      if (!(e = pipeline_event())) return cfail(c, RT_E_HIP, "rt_render_strips: events");
  }
  c->W = W;
  c->H = H;
  c->strip = strip;
  c->planned_batch = c->batch;
  return RT_OK;
}

// issue thread: for each handed-over slot, the gather half of the step on the gather stream
void issue_loop(rt_comm* c) {
  (void)hipSetDevice(c->device);
  using clk = std::chrono::steady_clock;
  while (true) {
    Job j;
    {
      // spin briefly for the next hand-over (a futex sleep + wake costs microseconds per step at frame
      // rates), then sleep until notified
      const uint64_t seen = c->done;
      const auto spin_end = clk::now() + std::chrono::microseconds(200);
      while (c->posted.load(std::memory_order_acquire) == seen && clk::now() < spin_end) __builtin_ia32_pause();
      std::unique_lock<std::mutex> lk(c->mu);
      c->sleeping.store(true, std::memory_order_seq_cst);
      c->cv_job.wait(lk, [c] { return c->stop || !c->jobs.empty(); });
      c->sleeping.store(false, std::memory_order_relaxed);
      if (c->aborting) c->jobs.clear();  // rt_comm_abort: no further collective
      if (c->jobs.empty()) return;  // stop requested and nothing left
      j = c->jobs.front();
      c->jobs.pop_front();
    }
    clk::time_point t0, t1, t2, t3;
    const clk::time_point tp0 = c->phase ? clk::now() : clk::time_point();
    if (c->timing) t0 = clk::now();
    Slot& s = c->slots[j.slot];
    rt_status st = RT_OK;
    std::string msg;
    if (j.rs != c->stream && hipStreamWaitEvent(c->stream, s.rendered, 0) != hipSuccess) {
      st = RT_E_HIP;
      msg = "rt_render_strips: render -> gather hand-off";
    }
    if (c->timing) t1 = clk::now();
    // the span starts once the gather stream is past the render (the wait above): the gather's own time, with any
    // wait for the other ranks' strips inside the collective
    hipEvent_t pa = st == RT_OK ? phase_begin(c, c->stream) : nullptr;
    if (st == RT_OK) {
      const size_t count = (size_t)j.nframes * j.rows_per_rank * j.W * kStripBpp;  // every frame of the slot, one call
      if (pa) {
        std::lock_guard<std::mutex> lk(c->pmu);
        c->p_bytes_in += (double)count * (c->nranks - 1);
        c->p_bytes += (double)count * c->nranks;
      }
      if (c->loopback) {
        // rank r's block (its first `count` bytes) to r x count in rank 0's buffer: ncclGather's layout
        const hipError_t e = hipMemcpy2DAsync(s.gathered, count, s.local, c->local_bytes, count, c->nranks,
                                              hipMemcpyDeviceToDevice, c->stream);
        if (e != hipSuccess) {
          st = RT_E_HIP;
          msg = std::string("rt_render_strips: loopback gather: ") + hipGetErrorString(e);
        }
      } else {
        ncclResult_t r =
            rccl().gather(s.local, c->rank == 0 ? s.gathered : nullptr, count, ncclUint8, 0, c->comm, c->stream);
        if (r != ncclSuccess) {
          st = RT_E_RCCL;
          msg = std::string("rt_render_strips: ncclGather: ") + rccl().getErrorString(r);
        }
      }
    }
    phase_end(c, c->stream, pa, kPhaseGather);
    if (c->timing) t2 = clk::now();
    // the gather's completion, for the step's tail on the slot's render stream (issue_tail_job, caller thread)
    if (st == RT_OK && j.rs != c->stream && hipEventRecord(s.gathered_ev, c->stream) != hipSuccess) {
      st = RT_E_HIP;
      msg = "rt_render_strips: record gather";
    }
    if (c->timing) {
      t3 = clk::now();
      c->w_parts[0] += std::chrono::duration<double, std::micro>(t1 - t0).count();
      c->w_parts[1] += std::chrono::duration<double, std::micro>(t2 - t1).count();
      c->w_parts[2] += std::chrono::duration<double, std::micro>(t3 - t2).count();
    }
    if (c->phase) {
      std::lock_guard<std::mutex> lk(c->pmu);
      c->p_issue_us += std::chrono::duration<double, std::micro>(clk::now() - tp0).count();
    }
    {
      std::lock_guard<std::mutex> lk(c->mu);
      if (st != RT_OK && c->werr == RT_OK) {
        c->werr = st;
        c->wmsg = msg;
      }
      c->done = j.seq;
    }
    c->cv_done.notify_all();
  }
}

// waits until the issue thread has enqueued every handed-over job up to `seq`
void wait_issued(rt_comm* c, uint64_t seq) {
  std::unique_lock<std::mutex> lk(c->mu);
  c->cv_done.wait(lk, [c, seq] { return c->done >= seq; });
}

rt_status worker_status(rt_comm* c);

// caller thread: a step's tail on its render stream, behind its gather (device-side wait): rank 0 assembles the
// frame there, off the gather stream, and the slot's next render on that stream follows it. A gather the issue
// thread failed to enqueue leaves its event stale: the assembly is skipped and the failure returned.
rt_status issue_tail_job(rt_comm* c, const Job& j) {
  wait_issued(c, j.seq);
  rt_status st = worker_status(c);
  if (st != RT_OK) return st;
  Slot& s = c->slots[j.slot];
  if (j.rs != c->stream && hipStreamWaitEvent(j.rs, s.gathered_ev, 0) != hipSuccess)
    return cfail(c, RT_E_HIP, "rt_render_strips: gather -> render stream hand-off");
  if (c->rank == 0) {
    // two assemblies into one frame buffer on different streams stay in call order
    for (Slot& o : c->slots) {
      if (&o == &s || !o.asm_stream || o.asm_stream == j.rs) continue;
      bool shared = false;
      for (uint32_t a = 0; a < o.asm_n; ++a)
        for (uint32_t b = 0; b < j.nframes; ++b) shared = shared || o.asm_frames[a] == j.frame_out[b];
      if (!shared) continue;
      if (hipEventRecord(o.asm_order, o.asm_stream) != hipSuccess || hipStreamWaitEvent(j.rs, o.asm_order, 0) != hipSuccess)
        return cfail(c, RT_E_HIP, "rt_render_strips: order after an assembly into the same frame");
    }
    // rank r's block of the gathered slot holds its strips of every frame in turn: frame b starts b frames into it;
    // the slot's frames are assembled by one launch
    const size_t frame_bytes = (size_t)j.rows_per_rank * j.W * kStripBpp;
    hipEvent_t pa = phase_begin(c, j.rs);
    const hipError_t e = rt::launch_assemble_frames(j.W, j.H, c->nranks, j.strip, s.gathered, j.frame_out, j.nframes,
                                                    frame_bytes, j.rs, j.nframes * j.rows_per_rank, kStripBpp);
    phase_end(c, j.rs, pa, kPhaseAssembly);
    if (e != hipSuccess) return cfail(c, RT_E_HIP, std::string("rt_render_strips: assembly: ") + hipGetErrorString(e));
    for (uint32_t b = 0; b < j.nframes; ++b) s.asm_frames[b] = j.frame_out[b];
    s.asm_stream = j.rs;
    s.asm_n = j.nframes;
  }
  // a frame issued on another stream than its slot's: its tail returns to that stream (rt_api.h)
  for (uint32_t b = 0; b < j.nframes; ++b) {
    if (!j.fs[b]) continue;
    if (hipEventRecord(s.fin[b], j.rs) != hipSuccess || hipStreamWaitEvent(j.fs[b], s.fin[b], 0) != hipSuccess)
      return cfail(c, RT_E_HIP, "rt_render_strips: tail -> the frame's render stream");
  }
  return RT_OK;
}

// issues the pending tails in call order: every one up to step `upto` (waiting for the issue thread where it is
// behind), then those whose gather the issue thread has already enqueued (no waiting)
rt_status issue_tails(rt_comm* c, uint64_t upto) {
  uint64_t done;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    done = c->done;
  }
  while (!c->tails.empty()) {
    const Job j = c->tails.front();
    if (j.seq > upto && j.seq > done) break;
    c->tails.pop_front();
    const rt_status st = issue_tail_job(c, j);
    if (st != RT_OK) return st;
  }
  return RT_OK;
}

// caller thread: the slot being filled is complete (its batch of frames, or fewer at a flush): the render event on
// its stream, then the gather half handed to the issue thread; its tail becomes pending
rt_status finish_slot(rt_comm* c) {
  if (c->fill == 0) return RT_OK;
  Job job = c->cur;
  job.nframes = c->fill;
  c->fill = 0;
  Slot& s = c->slots[job.slot];
  if (job.rs != c->stream && hipEventRecord(s.rendered, job.rs) != hipSuccess)
    return cfail(c, RT_E_HIP, "rt_render_strips: record render");
  s.used = true;
  s.last = job.rs;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    job.seq = ++c->issued;
    c->slot_seq[job.slot] = job.seq;
    c->jobs.push_back(job);
    c->posted.store(job.seq, std::memory_order_release);
  }
  if (c->sleeping.load(std::memory_order_seq_cst)) c->cv_job.notify_one();
  c->tails.push_back(job);
  return RT_OK;
}

rt_status worker_status(rt_comm* c) {
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->werr != RT_OK) {
    c->err = c->wmsg;
    return c->werr;
  }
  return RT_OK;
}

}  // namespace

extern "C" {

rt_status rt_comm_available(void) { return rccl().ok ? RT_OK : RT_E_UNSUPPORTED; }

rt_status rt_comm_get_unique_id(void* id_out) {
  if (!id_out) return RT_E_INVALID;
  RcclApi& api = rccl();
  if (!api.ok) return RT_E_UNSUPPORTED;
  ncclUniqueId id;
  if (api.getUniqueId(&id) != ncclSuccess) return RT_E_RCCL;
  static_assert(sizeof(ncclUniqueId) == RT_COMM_ID_BYTES, "ncclUniqueId size");
  std::memcpy(id_out, &id, sizeof(id));
  return RT_OK;
}

namespace {

// the communicator's streams, events and issue thread (no collective yet)
rt_comm* comm_create(rt_ctx_t ctx, uint32_t nranks, uint32_t rank, bool loopback) {
  rt_comm* c = new (std::nothrow) rt_comm();
  if (!c) return nullptr;
  c->ctx = ctx;
  c->device = rt::ctx_device(ctx);
  c->nranks = nranks;
  c->rank = rank;
  c->loopback = loopback;
  const char* tm = std::getenv("RT_COMM_TIMING");
  c->timing = tm && tm[0] == '1';
  // normal priority: a high-priority stream gets a hardware queue of its own (normal streams share
  // GPU_MAX_HW_QUEUES queues round robin, so a render stream can land on the gathers' queue), but its RCCL and
  // assembly kernels ran 3.5x / 4x slower there (tools/trace_share.py): not taken
  bool ok = hipSetDevice(c->device) == hipSuccess &&
            hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess;
  // one render stream (and pipeline slot) per hardware queue beside the gather stream's: GPU_MAX_HW_QUEUES is
  // HIP's queue count per process (4 by default); RT_COMM_SLOTS overrides (1..8)
  const char* hq = std::getenv("GPU_MAX_HW_QUEUES");
  const char* ns = std::getenv("RT_COMM_SLOTS");
  int queues = hq && std::atoi(hq) > 0 ? std::atoi(hq) : 4;
  int slots = ns && std::atoi(ns) > 0 ? std::atoi(ns) : queues - 1;
  c->nslots = (uint32_t)std::min<int>((int)kMaxSlots, std::max(1, slots));
  for (uint32_t k = 0; k < c->nslots; ++k)
    ok = ok && hipStreamCreateWithFlags(&c->rstreams[k], hipStreamNonBlocking) == hipSuccess;
  for (uint32_t k = 0; k < c->nslots; ++k) ok = ok && (c->join[k] = pipeline_event()) != nullptr;
  ok = ok && (c->xev = pipeline_event()) != nullptr;
  if (!ok) {
    for (hipStream_t& r : c->rstreams)
      if (r) (void)hipStreamDestroy(r);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    for (hipEvent_t& j : c->join)
      if (j) (void)hipEventDestroy(j);
    if (c->xev) (void)hipEventDestroy(c->xev);
    delete c;
    return nullptr;
  }
  return c;
}

void comm_free(rt_comm* c) {
  for (hipStream_t r : c->rstreams) {
    if (!r) continue;
    (void)hipStreamSynchronize(r);
    (void)rt::ctx_forget_stream(c->ctx, r);  // the context must not record on it at its next TLAS update
    (void)hipStreamDestroy(r);
  }
  if (c->stream) {
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamDestroy(c->stream);
  }
  release_slots(c);
  for (hipEvent_t j : c->join)
    if (j) (void)hipEventDestroy(j);
  if (c->xev) (void)hipEventDestroy(c->xev);
  for (const PhaseSpan& sp : c->ppend) {
    (void)hipEventDestroy(sp.a);
    (void)hipEventDestroy(sp.b);
  }
  for (hipEvent_t e : c->pfree) (void)hipEventDestroy(e);
  delete c;
}

}  // namespace

rt_status rt_comm_init(rt_ctx_t ctx, uint32_t nranks, uint32_t rank, const void* id, rt_comm_t* out) {
  if (!out) return RT_E_INVALID;
  *out = nullptr;
  if (!ctx || !id || nranks == 0 || rank >= nranks) return RT_E_INVALID;
  RcclApi& api = rccl();
  if (!api.ok) return RT_E_UNSUPPORTED;
  rt_comm* c = comm_create(ctx, nranks, rank, false);
  if (!c) return RT_E_HIP;
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  // collective: returns when every rank has joined
  if (api.commInitRank(&c->comm, (int)nranks, uid, (int)rank) != ncclSuccess) {
    c->comm = nullptr;
    comm_free(c);
    return RT_E_RCCL;
  }
  c->worker = std::thread(issue_loop, c);
  *out = c;
  return RT_OK;
}

rt_status rt_comm_init_loopback(rt_ctx_t ctx, uint32_t nranks, rt_comm_t* out) {
  if (!out) return RT_E_INVALID;
  *out = nullptr;
  if (!ctx || nranks == 0 || nranks > 64) return RT_E_INVALID;
  rt_comm* c = comm_create(ctx, nranks, 0, true);
  if (!c) return RT_E_HIP;
  c->worker = std::thread(issue_loop, c);
  *out = c;
  return RT_OK;
}

rt_status rt_comm_destroy(rt_comm_t c) {
  if (!c) return RT_E_INVALID;
  (void)hipSetDevice(c->device);
  // every step first, a partly filled slot included: its gather goes to the issue thread, which must still run
  const rt_status st = drain(c);
  {
    std::lock_guard<std::mutex> lk(c->mu);
    c->stop = true;
  }
  c->cv_job.notify_all();
  if (c->worker.joinable()) c->worker.join();  // the issue thread drains its queue first
  (void)hipSetDevice(c->device);
  if (c->timing && c->t_calls)
    std::fprintf(stderr, "rt_comm timing, caller thread (us per rt_render_strips over %llu calls): plan+checks %.2f, "
                 "render %.2f, record+hand-over %.2f, wait for the slot's last step %.2f, move to another stream %.2f, "
                 "previous step's tail %.2f\n", (unsigned long long)c->t_calls,
                 c->t_parts[0] / c->t_calls, c->t_parts[1] / c->t_calls, c->t_parts[2] / c->t_calls,
                 c->t_parts[3] / c->t_calls, c->t_parts[4] / c->t_calls, c->t_parts[5] / c->t_calls);
  if (c->timing && c->t_calls)
    std::fprintf(stderr, "rt_comm timing, issue thread (us per step): hand-off %.2f, ncclGather %.2f, gather event "
                 "%.2f\n", c->w_parts[0] / c->t_calls, c->w_parts[1] / c->t_calls, c->w_parts[2] / c->t_calls);
  if (c->comm) (void)rccl().commDestroy(c->comm);
  comm_free(c);
  return st;
}

// The failure path: no drain, no further collective. The caller thread's pending state (the slot being filled, the
// tails not yet issued) is dropped, the issue thread empties its queue and returns (a gather it is enqueuing right
// now completes its enqueue: RCCL calls return once enqueued), then ncclCommAbort cancels whatever the gather stream
// still waits on, so the stream synchronisations in comm_free return even when a peer never calls again.
rt_status rt_comm_abort(rt_comm_t c) {
  if (!c) return RT_E_INVALID;
  (void)hipSetDevice(c->device);
  c->fill = 0;
  c->tails.clear();
  {
    std::lock_guard<std::mutex> lk(c->mu);
    c->aborting = true;
    c->stop = true;
    c->jobs.clear();
  }
  c->cv_job.notify_all();
  if (c->worker.joinable()) c->worker.join();
  (void)hipSetDevice(c->device);
  rt_status st = RT_OK;
  if (c->comm) {
    RcclApi& api = rccl();
    const ncclResult_t r = api.commAbort ? api.commAbort(c->comm) : api.commDestroy(c->comm);
    if (r != ncclSuccess) st = RT_E_RCCL;
    c->comm = nullptr;
  }
  comm_free(c);
  return st;
}

const char* rt_comm_last_error(rt_comm_t c) { return c ? c->err.c_str() : "null communicator"; }

void* rt_comm_stream(rt_comm_t c) {
  if (!c) return nullptr;
  (void)hipSetDevice(c->device);
  if (finish_slot(c) != RT_OK || issue_tails(c, ~0ull) != RT_OK) return nullptr;
  wait_issued(c, c->issued);  // every step handed over so far is enqueued
  (void)hipSetDevice(c->device);
  // join: the stream returned (the gathers') waits, on the device, for the slots' render streams, where the
  // assemblies run
  hipStream_t seen[kMaxSlots];
  uint32_t k = 0;
  for (const Slot& s : c->slots) {
    if (!s.used || s.last == c->stream) continue;
    bool dup = false;
    for (uint32_t i = 0; i < k; ++i) dup = dup || seen[i] == s.last;
    if (dup) continue;
    if (hipEventRecord(c->join[k], s.last) != hipSuccess || hipStreamWaitEvent(c->stream, c->join[k], 0) != hipSuccess) {
      cfail(c, RT_E_HIP, "rt_comm_stream: join");
      return nullptr;
    }
    seen[k++] = s.last;
  }
  return (void*)c->stream;
}

uint32_t rt_comm_pipeline_depth(rt_comm_t c) { return c ? c->nslots * c->batch : 0; }

rt_status rt_comm_synchronize(rt_comm_t c) {
  if (!c) return RT_E_INVALID;
  (void)hipSetDevice(c->device);
  rt_status st = drain(c);
  if (st != RT_OK) return st;
  return worker_status(c);
}

rt_status rt_render_strips_frames(rt_comm_t c, uint32_t W, uint32_t H, uint32_t strip_rows, uint32_t nframes,
                                  const float* cameras, void* const* frames_out, void* render_stream) {
  if (!c) return RT_E_INVALID;
  if (W == 0 || H == 0 || strip_rows == 0) return cfail(c, RT_E_INVALID, "rt_render_strips: bad size");
  if (nframes == 0 || nframes > c->batch || nframes > (uint32_t)rt::kMaxLaunchFrames)
    return cfail(c, RT_E_INVALID, "rt_render_strips_frames: 1 .. rt_comm_batch frames per call");
  if (c->rank == 0) {
    bool ok = frames_out != nullptr;
    for (uint32_t b = 0; ok && b < nframes; ++b) ok = frames_out[b] != nullptr;
    if (!ok) return cfail(c, RT_E_INVALID, "rt_render_strips: rank 0 needs frame_out");
  }
  rt_status st = worker_status(c);
  if (st != RT_OK) return st;
  using clk = std::chrono::steady_clock;
  clk::time_point t0;
  const clk::time_point tp0 = c->phase ? clk::now() : clk::time_point();
  if (c->timing) t0 = clk::now();
  auto lap = [&](int part) {
    if (!c->timing) return;
    const clk::time_point t1 = clk::now();
    c->t_parts[part] += std::chrono::duration<double, std::micro>(t1 - t0).count();
    t0 = t1;
  };
  (void)hipSetDevice(c->device);
  // a new frame size, or frames that do not fit the slot being filled (one launch renders them: one slot): the
  // slot goes as it is
  if (c->fill && (c->W != W || c->H != H || c->strip != strip_rows || c->fill + nframes > c->batch)) {
    if ((st = finish_slot(c)) != RT_OK) return st;
  }
  if ((st = plan(c, W, H, strip_rows)) != RT_OK) return st;
  // every frame is validated (the scene may have changed since the slot's first frame)
  if (!c->rows.empty() && (st = rt::check_dispatch(c->ctx, W, H, c->slots[0].local, cameras != nullptr)) != RT_OK)
    return cfail(c, st, std::string("rt_render_strips: ") + rt_last_error(c->ctx));
  hipStream_t fs = nullptr;  // the caller's stream when it is not the slot's
  if (c->fill == 0) {  // a new slot: its first frame picks the render stream every frame of the slot uses
    const uint32_t si = (uint32_t)(c->next % c->nslots);
    hipStream_t rs = render_stream ? (hipStream_t)render_stream : c->rstreams[si];
    Slot& s = c->slots[si];
    ++c->next;
    lap(0);
    // the slot's previous frames must have left it: the tail of that step goes on the slot's stream first (waiting
    // for the issue thread to enqueue its gather, rarely: it keeps up), so a render on the same stream follows it in
    // stream order; a slot moved to another stream waits for it with an event
    if (s.used) {
      if ((st = issue_tails(c, c->slot_seq[si])) != RT_OK) return st;
      wait_issued(c, c->slot_seq[si]);
      lap(3);
      if (s.last != rs &&
          (hipEventRecord(s.moved, s.last) != hipSuccess || hipStreamWaitEvent(rs, s.moved, 0) != hipSuccess))
        return cfail(c, RT_E_HIP, "rt_render_strips: order after the slot's last step");
      lap(4);
    }
    c->cur = Job{};
    c->cur.slot = si;
    c->cur.rs = rs;
    c->cur.W = W;
    c->cur.H = H;
    c->cur.strip = strip_rows;
    c->cur.rows_per_rank = c->rows_per_rank;
  } else {
    lap(0);
    // a later frame of the slot issued on another stream: the slot's stream waits for the work the caller
    // queued there first (the frame's inputs); the tail comes back to it by an event (issue_tail_job)
    if (render_stream && (hipStream_t)render_stream != c->cur.rs) {
      fs = (hipStream_t)render_stream;
      if (hipEventRecord(c->xev, fs) != hipSuccess || hipStreamWaitEvent(c->cur.rs, c->xev, 0) != hipSuccess)
        return cfail(c, RT_E_HIP, "rt_render_strips: order after the frame's render stream");
    }
  }
  Slot& s = c->slots[c->cur.slot];
  // frames fill..fill+nframes-1 of the slot, one launch per rendered rank: frame b's strips b frames into the
  // rank's block, on the slot's render stream
  const uint64_t frame_bytes = (uint64_t)c->rows_per_rank * W * kStripBpp;
  hipEvent_t pa = phase_begin(c, c->cur.rs);
  uint32_t launches = 0;
  for (size_t r = 0; r < c->lb_count.size(); ++r) {
    if (!c->lb_count[r]) continue;  // a rank with no rows (H < nranks x strip_rows) renders nothing
    if (c->lb_render_count && (r < c->lb_render_first || r >= c->lb_render_first + c->lb_render_count)) continue;
    char* dst = (char*)s.local + r * c->local_bytes + (size_t)c->fill * frame_bytes;
    st = rt::dispatch_frame(c->ctx, W, H, c->d_rows + c->lb_first[r], c->lb_count[r], dst, nullptr, c->cur.rs,
                            kStripBpp, nframes, cameras, frame_bytes, c->rows_gen);
    if (st != RT_OK) return cfail(c, st, std::string("rt_render_strips: ") + rt_last_error(c->ctx));
    ++launches;
  }
  phase_end(c, c->cur.rs, pa, kPhaseRender);
  lap(1);
  for (uint32_t b = 0; b < nframes; ++b) {
    c->cur.frame_out[c->fill] = frames_out ? frames_out[b] : nullptr;
    c->cur.fs[c->fill] = fs;
    ++c->fill;
  }
  if (c->fill == c->batch && (st = finish_slot(c)) != RT_OK) return st;
  lap(2);
  // the tails whose gathers the issue thread has enqueued by now (no waiting)
  st = issue_tails(c, 0);
  lap(5);
  if (st != RT_OK) return st;
  ++c->t_calls;
  if (c->phase) {
    phase_collect(c, false);  // keeps the pending list short (host queries only)
    std::lock_guard<std::mutex> lk(c->pmu);
    c->p_frames += nframes;
    c->p_calls += 1;
    c->p_launches += launches;
    c->p_host_us += std::chrono::duration<double, std::micro>(clk::now() - tp0).count();
  }
  return RT_OK;
}

rt_status rt_render_strips(rt_comm_t c, uint32_t W, uint32_t H, uint32_t strip_rows, void* frame_out,
                           void* render_stream) {
  return rt_render_strips_frames(c, W, H, strip_rows, 1, nullptr, &frame_out, render_stream);
}

rt_status rt_comm_set_batch(rt_comm_t c, uint32_t frames_per_gather) {
  if (!c) return RT_E_INVALID;
  if (frames_per_gather == 0 || frames_per_gather > kMaxBatch)
    return cfail(c, RT_E_INVALID, "rt_comm_set_batch: 1 .. 4 frames per gather");
  if (frames_per_gather == c->batch) return RT_OK;
  (void)hipSetDevice(c->device);
  const rt_status st = drain(c);  // the slots are re-planned for the new size at the next frame
  if (st != RT_OK) return st;
  c->batch = frames_per_gather;
  return RT_OK;
}

uint32_t rt_comm_batch(rt_comm_t c) { return c ? c->batch : 0; }

rt_status rt_comm_set_phase_timing(rt_comm_t c, int on) {
  if (!c) return RT_E_INVALID;
  (void)hipSetDevice(c->device);
  const rt_status st = drain(c);  // the issue thread reads the flag: no step in flight when it changes
  if (st != RT_OK) return st;
  phase_reset(c);
  c->phase = on != 0;
  return RT_OK;
}

rt_status rt_comm_phase_stats(rt_comm_t c, double* out, uint32_t n) {
  if (!c || (!out && n)) return RT_E_INVALID;
  (void)hipSetDevice(c->device);
  const rt_status st = drain(c);  // every span recorded so far is on a stream that has drained
  if (st != RT_OK) return st;
  phase_collect(c, true);
  std::lock_guard<std::mutex> lk(c->pmu);
  const double v[RT_COMM_PHASE_COUNT] = {(double)c->p_frames, (double)c->p_launches, c->p_ms[kPhaseRender],
                                         (double)c->p_n[kPhaseGather], c->p_ms[kPhaseGather],
                                         (double)c->p_n[kPhaseAssembly], c->p_ms[kPhaseAssembly], c->p_host_us,
                                         (double)c->p_calls, c->p_issue_us, c->p_bytes_in, c->p_bytes};
  std::memcpy(out, v, std::min<uint32_t>(n, RT_COMM_PHASE_COUNT) * sizeof(double));
  return RT_OK;
}

rt_status rt_comm_loopback_render_ranks(rt_comm_t c, uint32_t first, uint32_t count) {
  if (!c) return RT_E_INVALID;
  if (!c->loopback) return cfail(c, RT_E_INVALID, "rt_comm_loopback_render_ranks: loopback communicators only");
  if (count && (first >= c->nranks || count > c->nranks - first))
    return cfail(c, RT_E_INVALID, "rt_comm_loopback_render_ranks: ranks out of range");
  c->lb_render_first = count ? first : 0;
  c->lb_render_count = count;
  return RT_OK;
}

}  // extern "C"
