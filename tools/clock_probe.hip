// Where the tile balance's recording kernel gets its extra HBM reads (the BAL instantiation fetches
// ~9 MB per 1080p launch more than the plain kernel, on C2F and C4 alike, i.e. per wave, not per scene). Each wave of
// these kernels does what the recording kernel does around its walk except the walk: read a clock at its start and
// at its end, and lane 0 stores the difference into a per-wave word (the cost map's layout: 2 words per wave slot).
// KIND 0 stores a constant (no clock), 1 reads s_memrealtime (the 100 MHz "real time" counter, the shipped
// recording), 2 reads s_memtime (the shader-clock counter), 3 s_memrealtime at the start only. Run under
//   rocprofv3 --pmc FETCH_SIZE -- tools/bin/clock_probe
// with 32,400 waves per launch (a 1080p frame's 8 x 8 tiles); the FETCH_SIZE difference between the kinds is what
// the clock reads cost in fabric traffic.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

template <int KIND>
__global__ __launch_bounds__(128) void k_clock(uint32_t* cost, uint32_t spin) {
  const uint32_t w = blockIdx.x * 2u + (threadIdx.x >> 6);
  uint64_t t0 = 0;
  if (KIND == 1 || KIND == 3) t0 = __builtin_amdgcn_s_memrealtime();
  if (KIND == 2) t0 = __builtin_amdgcn_s_memtime();
  // a little VALU work in place of the walk (keeps the wave resident a while)
  float x = (float)threadIdx.x;
  for (uint32_t i = 0; i < spin; ++i) x = __builtin_fmaf(x, 1.0000001f, 0.5f);
  uint32_t dt = x > 1e30f ? 1u : 0u;
  if (KIND == 1) dt += (uint32_t)(__builtin_amdgcn_s_memrealtime() - t0);
  if (KIND == 2) dt += (uint32_t)(__builtin_amdgcn_s_memtime() - t0);
  if (KIND == 3) dt += (uint32_t)t0;
  if ((threadIdx.x & 63u) == 0u) cost[2u * w] = dt;
}

int main() {
  const uint32_t waves = 32400, blocks = waves / 2;
  uint32_t* cost = nullptr;
  if (hipMalloc(&cost, waves * 8) != hipSuccess) return 1;
  (void)hipMemset(cost, 0, waves * 8);
  for (int rep = 0; rep < 5; ++rep) {
    hipLaunchKernelGGL(k_clock<0>, dim3(blocks), dim3(128), 0, 0, cost, 2000u);
    hipLaunchKernelGGL(k_clock<1>, dim3(blocks), dim3(128), 0, 0, cost, 2000u);
    hipLaunchKernelGGL(k_clock<2>, dim3(blocks), dim3(128), 0, 0, cost, 2000u);
    hipLaunchKernelGGL(k_clock<3>, dim3(blocks), dim3(128), 0, 0, cost, 2000u);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  uint32_t h[4];
  (void)hipMemcpy(h, cost, sizeof(h), hipMemcpyDeviceToHost);
  std::printf("{\"waves\": %u, \"last_cost\": [%u, %u]}\n", waves, h[0], h[2]);
  (void)hipFree(cost);
  return 0;
}
