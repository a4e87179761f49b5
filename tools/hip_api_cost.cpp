// Host cost of the HIP runtime calls one tiled-frame step makes (rt_render_strips and its issue thread), each
// timed over many back-to-back calls while the GPU is kept busy (a long kernel queued first, so no call waits
// for an idle device):
//   hipcc --offload-arch=gfx950 -O2 -o gpurun_out/hip_api_cost tools/hip_api_cost.cpp && gpurun_out/hip_api_cost
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void k_spin(unsigned long long cycles) {
  const unsigned long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
}
__global__ void k_empty(int* p) {
  if (p && threadIdx.x == 1023) p[0] = 1;
}

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));      \
      return 1;                                                          \
    }                                                                    \
  } while (0)

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) {
  return std::chrono::duration<double, std::micro>(b - a).count();
}

int main() {
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t ev[8];
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence));
  int* d = nullptr;
  CK(hipMalloc(&d, 4));
  // warm up
  for (int i = 0; i < 100; ++i) k_empty<<<2048, 256, 0, s0>>>(d);
  CK(hipDeviceSynchronize());
  // each section: both streams busy behind a spin kernel (~0.05-1 s), then n calls timed on the host; n stays
  // well below the hardware queue's packet capacity so no call waits for queue space
  const int n = 300;
  auto section = [&](auto fn) -> double {
    k_spin<<<1, 64, 0, s0>>>(100000000ull);
    k_spin<<<1, 64, 0, s1>>>(100000000ull);
    const auto t0 = clk::now();
    for (int i = 0; i < n; ++i) fn(i);
    const double r = us(t0, clk::now()) / n;
    (void)hipDeviceSynchronize();
    return r;
  };
  const double launch = section([&](int) { k_empty<<<2048, 256, 0, s0>>>(d); });
  const double record = section([&](int i) { (void)hipEventRecord(ev[i & 7], s0); });
  const double wait = section([&](int i) { (void)hipStreamWaitEvent(s1, ev[i & 7], 0); });
  const double query = section([&](int i) { (void)hipEventQuery(ev[i & 7]); });
  const double setdev = section([&](int) { (void)hipSetDevice(0); });
  const double step = section([&](int i) {
    (void)hipStreamWaitEvent(s0, ev[(i + 4) & 7], 0);
    k_empty<<<2048, 256, 0, s0>>>(d);
    (void)hipEventRecord(ev[i & 7], s0);
  });
  std::printf("{\"launch_us\": %.3f, \"event_record_us\": %.3f, \"stream_wait_event_us\": %.3f, \"event_query_us\": %.3f, "
              "\"set_device_us\": %.3f, \"wait_launch_record_us\": %.3f, \"calls\": %d}\n",
              launch, record, wait, query, setdev, step, n);
  return 0;
}
