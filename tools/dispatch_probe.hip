// Probe kernels for tools/queue_probe.py: which of k_tile_plan's resources — 16 waves of one
// workgroup on one CU, 135 KB of LDS — makes it wait ~60 us to start beside trace frames. Each kernel is one
// workgroup that stamps its start (s_memrealtime) and does a few microseconds of work:
//   kind 0: 1024 threads, 135 KB LDS (k_tile_plan's shape)   kind 1: 1024 threads, no LDS
//   kind 2: 256 threads, 135 KB LDS                          kind 3: 256 threads, no LDS
// Built by the Makefile into tools/bin/libdispatch_probe.so; launched through ctypes on the caller's stream.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr uint32_t kWords = 34000;  // 136 KB of LDS

template <uint32_t THREADS, bool LDS>
__global__ __launch_bounds__(THREADS) void k_probe(uint32_t* out) {
  __shared__ uint32_t s[LDS ? kWords : 1];
  uint32_t acc = threadIdx.x;
  if (LDS) {
    for (uint32_t i = threadIdx.x; i < kWords; i += THREADS) s[i] = i * 3u;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < kWords; i += THREADS) acc += s[(i * 7u) % kWords];
  } else {
    for (uint32_t i = 0; i < 64; ++i) acc = acc * 1664525u + 1013904223u;
  }
  if (threadIdx.x == 0) out[0] = acc;
}

}  // namespace

extern "C" int dispatch_probe(int kind, uint32_t* out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  switch (kind) {
    case 0: hipLaunchKernelGGL((k_probe<1024, true>), dim3(1), dim3(1024), 0, s, out); break;
    case 1: hipLaunchKernelGGL((k_probe<1024, false>), dim3(1), dim3(1024), 0, s, out); break;
    case 2: hipLaunchKernelGGL((k_probe<256, true>), dim3(1), dim3(256), 0, s, out); break;
    case 3: hipLaunchKernelGGL((k_probe<256, false>), dim3(1), dim3(256), 0, s, out); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
