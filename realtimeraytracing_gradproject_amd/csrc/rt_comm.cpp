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
// RCCL is bound at run time (dlopen of librccl.so.1): a process that already loaded RCCL (torch)
// shares that copy, and a context that never creates a communicator never loads it.
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
    api.gather = (decltype(api.gather))sym("ncclGather");
    api.getErrorString = (decltype(api.getErrorString))sym("ncclGetErrorString");
    api.ok = api.getUniqueId && api.commInitRank && api.commDestroy && api.gather && api.getErrorString;
    if (!api.ok) api.err = "librccl.so.1 lacks ncclGather / ncclCommInitRank";
  });
  return api;
}

// frames per gather (rt_comm_set_batch): a slot holds up to this many consecutive frames' strips
constexpr uint32_t kMaxBatch = 4;

struct Slot {
  void* local = nullptr;     // this rank's strips, compact: batch x rows_per_rank x W RGBA8 (frame-major)
  void* gathered = nullptr;  // rank 0: nranks x (batch x rows_per_rank) x W RGBA8 (rank-major, as ncclGather lays it)
  hipEvent_t rendered = nullptr;  // on the slot's render stream, after its render
  hipEvent_t gathered_ev = nullptr;  // on the gather stream, after its gather
  hipEvent_t moved = nullptr;     // recorded on demand (a slot moved to another stream)
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

struct Job {
  uint32_t slot;
  uint32_t nframes;                // frames in the slot (their strips are gathered by one ncclGather)
  void* frame_out[kMaxBatch];      // rank 0's output frame of each
  hipStream_t rs;  // the slot's render stream: its assembly runs there
  uint32_t W, H, strip, rows_per_rank;
  uint64_t seq;
};

struct rt_comm {
  rt_ctx_t ctx = nullptr;
  int device = 0;
  uint32_t nranks = 1, rank = 0;
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
  std::vector<uint32_t> rows;  // this rank's global rows, output order
  uint32_t* d_rows = nullptr;  // ... on the device (uploaded once per plan)
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
  rt_status werr = RT_OK;       // the issue thread's first failure, returned by the next call
  std::string wmsg;
  double w_parts[3] = {0, 0, 0};  // RT_COMM_TIMING: issue-thread hand-off, ncclGather, gather event
};

namespace {

rt_status cfail(rt_comm* c, rt_status st, const std::string& m) {
  if (c) c->err = m;
  return st;
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
  const uint32_t n = rt_strip_rows(H, c->nranks, c->rank, strip, nullptr, 0);
  c->rows.assign(n, 0u);
  if (n) rt_strip_rows(H, c->nranks, c->rank, strip, c->rows.data(), n);
  if (n) {
    if (hipMalloc(&c->d_rows, (size_t)n * 4) != hipSuccess) return cfail(c, RT_E_OOM, "rt_render_strips: hipMalloc(rows)");
    if (hipMemcpy(c->d_rows, c->rows.data(), (size_t)n * 4, hipMemcpyHostToDevice) != hipSuccess)
      return cfail(c, RT_E_HIP, "rt_render_strips: upload rows");
  }
  const uint32_t nstrips = (H + strip - 1) / strip;
  c->rows_per_rank = ((nstrips + c->nranks - 1) / c->nranks) * strip;
  const size_t local_bytes = (size_t)c->rows_per_rank * W * 4 * c->batch;
  for (uint32_t k = 0; k < c->nslots; ++k) {
    Slot& s = c->slots[k];
    if (hipMalloc(&s.local, local_bytes) != hipSuccess) return cfail(c, RT_E_OOM, "rt_render_strips: hipMalloc(local)");
    if (c->rank == 0 && hipMalloc(&s.gathered, local_bytes * c->nranks) != hipSuccess)
      return cfail(c, RT_E_OOM, "rt_render_strips: hipMalloc(gathered)");
    if (!(s.rendered = pipeline_event()) || !(s.gathered_ev = pipeline_event()) || !(s.moved = pipeline_event()) ||
        !(s.asm_order = pipeline_event()))
      return cfail(c, RT_E_HIP, "rt_render_strips: events");
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
      if (c->jobs.empty()) return;  // stop requested and nothing left
      j = c->jobs.front();
      c->jobs.pop_front();
    }
    clk::time_point t0, t1, t2, t3;
    if (c->timing) t0 = clk::now();
    Slot& s = c->slots[j.slot];
    rt_status st = RT_OK;
    std::string msg;
    if (j.rs != c->stream && hipStreamWaitEvent(c->stream, s.rendered, 0) != hipSuccess) {
      st = RT_E_HIP;
      msg = "rt_render_strips: render -> gather hand-off";
    }
    if (c->timing) t1 = clk::now();
    if (st == RT_OK) {
      const size_t count = (size_t)j.nframes * j.rows_per_rank * j.W * 4;  // every frame of the slot, one call
      ncclResult_t r = rccl().gather(s.local, c->rank == 0 ? s.gathered : nullptr, count, ncclUint8, 0, c->comm, c->stream);
      if (r != ncclSuccess) {
        st = RT_E_RCCL;
        msg = std::string("rt_render_strips: ncclGather: ") + rccl().getErrorString(r);
      }
    }
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

// caller thread: a step's tail on its render stream, behind its gather (device-side wait): rank 0 assembles the
// frame there, off the gather stream, and the slot's next render on that stream follows it
rt_status issue_tail_job(rt_comm* c, const Job& j) {
  wait_issued(c, j.seq);
  Slot& s = c->slots[j.slot];
  if (j.rs != c->stream && hipStreamWaitEvent(j.rs, s.gathered_ev, 0) != hipSuccess)
    return cfail(c, RT_E_HIP, "rt_render_strips: gather -> render stream hand-off");
  if (c->rank != 0) return RT_OK;
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
  // rank r's block of the gathered slot holds its strips of every frame in turn: frame b starts b frames into it
  const size_t frame_bytes = (size_t)j.rows_per_rank * j.W * 4;
  for (uint32_t b = 0; b < j.nframes; ++b) {
    const hipError_t e = rt::launch_assemble_strips(j.W, j.H, c->nranks, j.strip, (const char*)s.gathered + b * frame_bytes,
                                                    j.frame_out[b], j.rs, j.nframes * j.rows_per_rank);
    if (e != hipSuccess) return cfail(c, RT_E_HIP, std::string("rt_render_strips: assembly: ") + hipGetErrorString(e));
    s.asm_frames[b] = j.frame_out[b];
  }
  s.asm_stream = j.rs;
  s.asm_n = j.nframes;
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

rt_status rt_comm_init(rt_ctx_t ctx, uint32_t nranks, uint32_t rank, const void* id, rt_comm_t* out) {
  if (!out) return RT_E_INVALID;
  *out = nullptr;
  if (!ctx || !id || nranks == 0 || rank >= nranks) return RT_E_INVALID;
  RcclApi& api = rccl();
  if (!api.ok) return RT_E_UNSUPPORTED;
  rt_comm* c = new (std::nothrow) rt_comm();
  if (!c) return RT_E_OOM;
  c->ctx = ctx;
  c->device = rt::ctx_device(ctx);
  c->nranks = nranks;
  c->rank = rank;
  const char* tm = std::getenv("RT_COMM_TIMING");
  c->timing = tm && tm[0] == '1';
  // normal priority: a high-priority stream gets a hardware queue of its own (normal streams share
  // GPU_MAX_HW_QUEUES queues round robin, so a render stream can land on the gathers' queue), but its RCCL and
  // assembly kernels ran 3.5x / 4x slower there (tools/trace_share.py): not taken
  auto destroy_streams = [c]() {
    for (hipStream_t& r : c->rstreams)
      if (r) (void)hipStreamDestroy(r);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    for (hipEvent_t& j : c->join)
      if (j) (void)hipEventDestroy(j);
  };
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
  if (!ok) {
    destroy_streams();
    delete c;
    return RT_E_HIP;
  }
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  // collective: returns when every rank has joined
  if (api.commInitRank(&c->comm, (int)nranks, uid, (int)rank) != ncclSuccess) {
    destroy_streams();
    delete c;
    return RT_E_RCCL;
  }
  c->worker = std::thread(issue_loop, c);
  *out = c;
  return RT_OK;
}

rt_status rt_comm_destroy(rt_comm_t c) {
  if (!c) return RT_E_INVALID;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    c->stop = true;
  }
  c->cv_job.notify_all();
  if (c->worker.joinable()) c->worker.join();  // the issue thread drains its queue first
  (void)hipSetDevice(c->device);
  (void)drain(c);
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
  release_slots(c);
  for (hipStream_t r : c->rstreams) {
    if (!r) continue;
    (void)hipStreamSynchronize(r);
    (void)hipStreamDestroy(r);
  }
  (void)hipStreamDestroy(c->stream);
  for (hipEvent_t j : c->join)
    if (j) (void)hipEventDestroy(j);
  delete c;
  return RT_OK;
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

rt_status rt_render_strips(rt_comm_t c, uint32_t W, uint32_t H, uint32_t strip_rows, void* frame_out,
                           void* render_stream) {
  if (!c) return RT_E_INVALID;
  if (W == 0 || H == 0 || strip_rows == 0) return cfail(c, RT_E_INVALID, "rt_render_strips: bad size");
  if (c->rank == 0 && !frame_out) return cfail(c, RT_E_INVALID, "rt_render_strips: rank 0 needs frame_out");
  rt_status st = worker_status(c);
  if (st != RT_OK) return st;
  using clk = std::chrono::steady_clock;
  clk::time_point t0;
  if (c->timing) t0 = clk::now();
  auto lap = [&](int part) {
    if (!c->timing) return;
    const clk::time_point t1 = clk::now();
    c->t_parts[part] += std::chrono::duration<double, std::micro>(t1 - t0).count();
    t0 = t1;
  };
  (void)hipSetDevice(c->device);
  if (c->fill && (c->W != W || c->H != H || c->strip != strip_rows)) {
    if ((st = finish_slot(c)) != RT_OK) return st;  // a new frame size: the slot being filled goes as it is
  }
  if ((st = plan(c, W, H, strip_rows)) != RT_OK) return st;
  // every frame is validated (the scene may have changed since the slot's first frame)
  if (!c->rows.empty() && (st = rt::check_dispatch(c->ctx, W, H, c->slots[0].local)) != RT_OK)
    return cfail(c, st, std::string("rt_render_strips: ") + rt_last_error(c->ctx));
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
    c->cur = Job{si, 0, {}, rs, W, H, strip_rows, c->rows_per_rank, 0};
  } else {
    lap(0);
  }
  Slot& s = c->slots[c->cur.slot];
  if (!c->rows.empty()) {
    // frame b of the slot: its strips b frames into the slot's buffer, on the slot's render stream
    char* dst = (char*)s.local + (size_t)c->fill * c->rows_per_rank * W * 4;
    st = rt::dispatch_frame(c->ctx, W, H, c->d_rows, (uint32_t)c->rows.size(), dst, nullptr, c->cur.rs);
    if (st != RT_OK) return cfail(c, st, std::string("rt_render_strips: ") + rt_last_error(c->ctx));
  }
  lap(1);
  c->cur.frame_out[c->fill++] = frame_out;
  if (c->fill == c->batch && (st = finish_slot(c)) != RT_OK) return st;
  lap(2);
  // the tails whose gathers the issue thread has enqueued by now (no waiting)
  st = issue_tails(c, 0);
  lap(5);
  if (st != RT_OK) return st;
  ++c->t_calls;
  return RT_OK;
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

}  // extern "C"
