// rt_comm.cpp — the multi-GPU frame loop behind the C-ABI: one frame tiled over the
// ranks in interleaved strips, ONE ncclGather of every rank's compact strip buffer into rank 0
// (rccl.h:745), then the un-interleave kernel (rt_assemble_strips) on rank 0. One process per GPU,
// each with its own rt_ctx and the full scene; nothing but finished strips crosses xGMI.
//
// The frame being tiled is the reference's DispatchRays W x H (D3D12HelloTriangle.cpp:584-592),
// issued once per OnRender (:436-471). The whole step is issued from C++ (render on the caller's
// stream, gather + assembly on the communicator's stream, device-side events between them), so a
// step costs one call of host issue instead of a Python loop of collectives.
//
// RCCL is bound at run time (dlopen of librccl.so.1): a process that already loaded RCCL (torch)
// shares that copy, and a context that never creates a communicator never loads it.
//
// Two host threads issue a step: the caller's thread renders (wait for the slot, dispatch, record the
// render event) and hands the slot to the communicator's issue thread, which orders the gather after
// the render, issues the ncclGather and the assembly and records the slot's release. HIP and RCCL host
// calls cost microseconds each, so one thread issuing both halves limited a step to their sum (≈ 26 us
// measured, tools/native_strips_cost.py); split, a step costs the longer half.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

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

struct Slot {
  void* local = nullptr;     // this rank's strips, compact: rows_per_rank x W RGBA8
  void* gathered = nullptr;  // rank 0: nranks x rows_per_rank x W RGBA8
  hipEvent_t rendered = nullptr, freed = nullptr;
  bool used = false;
};

constexpr uint32_t kSlots = 4;  // frames in the render -> gather pipeline (frames in flight <= 4, bench.py)

hipEvent_t pipeline_event() {
  hipEvent_t e = nullptr;
  // device-side hand-offs only: no timestamp, no system-scope release (rt_event_create's flags)
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess) return nullptr;
  return e;
}

}  // namespace

struct Job {
  uint32_t slot;
  void* frame_out;
  uint32_t W, H, strip, rows_per_rank;
  uint64_t seq;
};

struct rt_comm {
  rt_ctx_t ctx = nullptr;
  int device = 0;
  uint32_t nranks = 1, rank = 0;
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;  // gathers + assembly
  // the communicator's own render streams (render_stream NULL: slot k renders on rstreams[k % kRenderStreams]),
  // created right after `stream`, so the four take four different hardware queues (HIP deals a process's
  // streams over GPU_MAX_HW_QUEUES = 4 queues in creation order): no render shares the gathers' queue
  hipStream_t rstreams[3] = {nullptr, nullptr, nullptr};
  std::string err;
  // frame geometry of the slots (re-planned when it changes)
  uint32_t W = 0, H = 0, strip = 0, rows_per_rank = 0;
  std::vector<uint32_t> rows;  // this rank's global rows, output order
  uint32_t* d_rows = nullptr;  // ... on the device (uploaded once per plan)
  // RT_COMM_TIMING=1 (diagnostics): host time per part of rt_render_strips, printed by rt_comm_destroy
  bool timing = false;
  double t_parts[5] = {0, 0, 0, 0, 0};
  uint64_t t_calls = 0;
  Slot slots[kSlots];
  uint64_t next = 0;
  // the issue thread of the gather side (see the header comment)
  std::thread worker;
  std::mutex mu;
  std::condition_variable cv_job, cv_done;
  std::deque<Job> jobs;
  uint64_t issued = 0;          // jobs handed over (caller thread)
  uint64_t done = 0;            // jobs whose gather, assembly and release are enqueued (issue thread)
  uint64_t slot_seq[kSlots] = {0, 0, 0, 0};  // the last job of each slot
  bool stop = false;
  rt_status werr = RT_OK;       // the issue thread's first failure, returned by the next call
  std::string wmsg;
  double w_parts[3] = {0, 0, 0};  // RT_COMM_TIMING: issue-thread hand-off, ncclGather, assembly + record
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
    if (s.rendered) (void)hipEventDestroy(s.rendered);
    if (s.freed) (void)hipEventDestroy(s.freed);
    s = Slot();
  }
}

// (re)plans the strips of a W x H frame and sizes the pipeline slots; waits for the slots' last uses
void wait_issued(rt_comm* c, uint64_t seq);

rt_status plan(rt_comm* c, uint32_t W, uint32_t H, uint32_t strip) {
  if (c->W == W && c->H == H && c->strip == strip) return RT_OK;
  wait_issued(c, c->issued);
  if (c->stream && hipStreamSynchronize(c->stream) != hipSuccess) return cfail(c, RT_E_HIP, "rt_render_strips: drain");
  for (Slot& s : c->slots)
    if (s.used && s.freed && hipEventSynchronize(s.freed) != hipSuccess)
      return cfail(c, RT_E_HIP, "rt_render_strips: drain");
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
  const size_t local_bytes = (size_t)c->rows_per_rank * W * 4;
  for (Slot& s : c->slots) {
    if (hipMalloc(&s.local, local_bytes) != hipSuccess) return cfail(c, RT_E_OOM, "rt_render_strips: hipMalloc(local)");
    if (c->rank == 0 && hipMalloc(&s.gathered, local_bytes * c->nranks) != hipSuccess)
      return cfail(c, RT_E_OOM, "rt_render_strips: hipMalloc(gathered)");
    if (!(s.rendered = pipeline_event()) || !(s.freed = pipeline_event()))
      return cfail(c, RT_E_HIP, "rt_render_strips: events");
  }
  c->W = W;
  c->H = H;
  c->strip = strip;
  return RT_OK;
}

// issue thread: for each handed-over slot, the gather side of the step on the communicator's stream
void issue_loop(rt_comm* c) {
  (void)hipSetDevice(c->device);
  using clk = std::chrono::steady_clock;
  while (true) {
    Job j;
    {
      std::unique_lock<std::mutex> lk(c->mu);
      c->cv_job.wait(lk, [c] { return c->stop || !c->jobs.empty(); });
      if (c->jobs.empty()) return;  // stop requested and nothing left
      j = c->jobs.front();
      c->jobs.pop_front();
    }
    clk::time_point t0, t1, t2, t3;
    if (c->timing) t0 = clk::now();
    Slot& s = c->slots[j.slot];
    rt_status st = RT_OK;
    std::string msg;
    if (hipStreamWaitEvent(c->stream, s.rendered, 0) != hipSuccess) {
      st = RT_E_HIP;
      msg = "rt_render_strips: render -> gather hand-off";
    }
    if (c->timing) t1 = clk::now();
    if (st == RT_OK) {
      const size_t count = (size_t)j.rows_per_rank * j.W * 4;
      ncclResult_t r = rccl().gather(s.local, c->rank == 0 ? s.gathered : nullptr, count, ncclUint8, 0, c->comm, c->stream);
      if (r != ncclSuccess) {
        st = RT_E_RCCL;
        msg = std::string("rt_render_strips: ncclGather: ") + rccl().getErrorString(r);
      }
    }
    if (c->timing) t2 = clk::now();
    if (st == RT_OK && c->rank == 0) {
      // the launcher itself, not rt_assemble_strips: the caller's thread owns the context's state
      const hipError_t e = rt::launch_assemble_strips(j.W, j.H, c->nranks, j.strip, s.gathered, j.frame_out, c->stream);
      if (e != hipSuccess) {
        st = RT_E_HIP;
        msg = std::string("rt_render_strips: assembly: ") + hipGetErrorString(e);
      }
    }
    if (st == RT_OK && hipEventRecord(s.freed, c->stream) != hipSuccess) {
      st = RT_E_HIP;
      msg = "rt_render_strips: record";
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
  };
  bool ok = hipSetDevice(c->device) == hipSuccess &&
            hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess;
  for (hipStream_t& r : c->rstreams) ok = ok && hipStreamCreateWithFlags(&r, hipStreamNonBlocking) == hipSuccess;
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
  (void)hipStreamSynchronize(c->stream);
  for (Slot& s : c->slots)
    if (s.used && s.freed) (void)hipEventSynchronize(s.freed);
  if (c->timing && c->t_calls)
    std::fprintf(stderr, "rt_comm timing, caller thread (us per rt_render_strips over %llu calls): plan+checks %.2f, "
                 "render %.2f, record+hand-over %.2f, wait for the slot's hand-off %.2f, stream wait %.2f\n",
                 (unsigned long long)c->t_calls,
                 c->t_parts[0] / c->t_calls, c->t_parts[1] / c->t_calls, c->t_parts[2] / c->t_calls,
                 c->t_parts[3] / c->t_calls, c->t_parts[4] / c->t_calls);
  if (c->timing && c->t_calls)
    std::fprintf(stderr, "rt_comm timing, issue thread (us per step): hand-off %.2f, ncclGather %.2f, assembly+record "
                 "%.2f\n", c->w_parts[0] / c->t_calls, c->w_parts[1] / c->t_calls, c->w_parts[2] / c->t_calls);
  if (c->comm) (void)rccl().commDestroy(c->comm);
  release_slots(c);
  for (hipStream_t r : c->rstreams) {
    (void)hipStreamSynchronize(r);
    (void)hipStreamDestroy(r);
  }
  (void)hipStreamDestroy(c->stream);
  delete c;
  return RT_OK;
}

const char* rt_comm_last_error(rt_comm_t c) { return c ? c->err.c_str() : "null communicator"; }

void* rt_comm_stream(rt_comm_t c) {
  if (!c) return nullptr;
  wait_issued(c, c->issued);  // every step handed over so far is enqueued on the stream returned
  return (void*)c->stream;
}

rt_status rt_comm_synchronize(rt_comm_t c) {
  if (!c) return RT_E_INVALID;
  wait_issued(c, c->issued);
  (void)hipSetDevice(c->device);
  rt_status st = worker_status(c);
  if (st != RT_OK) return st;
  return hipStreamSynchronize(c->stream) == hipSuccess ? RT_OK : cfail(c, RT_E_HIP, "rt_comm_synchronize");
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
  if ((st = plan(c, W, H, strip_rows)) != RT_OK) return st;
  const uint32_t si = (uint32_t)(c->next % kSlots);
  hipStream_t rs = render_stream ? (hipStream_t)render_stream : c->rstreams[si % 3];
  Slot& s = c->slots[si];
  if (!c->rows.empty() && (st = rt::check_dispatch(c->ctx, W, H, s.local)) != RT_OK)
    return cfail(c, st, std::string("rt_render_strips: ") + rt_last_error(c->ctx));
  ++c->next;
  lap(0);
  // the slot's previous frame must have left it: its release is recorded by the issue thread (wait for
  // that, rarely: four slots), then this stream waits for it on the device
  if (s.used) {
    wait_issued(c, c->slot_seq[si]);
    lap(3);
    if (hipStreamWaitEvent(rs, s.freed, 0) != hipSuccess)
      return cfail(c, RT_E_HIP, "rt_render_strips: order after the slot's last gather");
    lap(4);
  }
  if (!c->rows.empty()) {
    st = rt::dispatch_frame(c->ctx, W, H, c->d_rows, (uint32_t)c->rows.size(), s.local, nullptr, rs);
    if (st != RT_OK) return cfail(c, st, std::string("rt_render_strips: ") + rt_last_error(c->ctx));
  }
  lap(1);
  if (hipEventRecord(s.rendered, rs) != hipSuccess) return cfail(c, RT_E_HIP, "rt_render_strips: record render");
  s.used = true;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    const uint64_t seq = ++c->issued;
    c->slot_seq[si] = seq;
    c->jobs.push_back(Job{si, frame_out, W, H, strip_rows, c->rows_per_rank, seq});
  }
  c->cv_job.notify_one();
  lap(2);
  ++c->t_calls;
  return RT_OK;
}

}  // extern "C"
