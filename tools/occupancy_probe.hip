// Resident waves per SIMD on this GPU (the trace kernel's wave-time traces never exceed 7 waves per
// SIMD although the compiler and hipOccupancyMaxActiveBlocksPerMultiprocessor report 8). Each probe kernel's waves
// spin for a fixed time and record (start, end) clocks and their HW_ID; the host sweeps the events per SIMD and
// reports the most waves ever resident on one SIMD. Kernels differ only in the registers they hold (an asm clobber
// of the highest VGPR / SGPR forces the allocation), at the trace kernel's 128-thread workgroups.
//   tools/bin/occupancy_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <map>
#include <utility>
#include <vector>

#define CLOB_V(n) asm volatile("v_mov_b32 v" #n ", 0" ::: "v" #n)
#define CLOB_S(n) asm volatile("s_mov_b32 s" #n ", 0" ::: "s" #n)

template <int KIND, int BLOCK = 128>
__global__ __launch_bounds__(BLOCK) void k_probe(uint4* rec, uint32_t spin_ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  if (KIND == 1) CLOB_V(60);           // 61 VGPRs (the trace kernel's 57..61)
  if (KIND == 2) CLOB_V(63);           // 64 VGPRs
  if (KIND == 3) CLOB_V(64);           // 65 VGPRs (-> 7 waves by VGPRs)
  if (KIND == 4) { CLOB_V(60); CLOB_S(87); }   // 61 VGPRs + 88 SGPRs (the trace kernel's descriptor)
  if (KIND == 5) { CLOB_V(8); CLOB_S(99); }    // few VGPRs, 100 SGPRs
  if (KIND == 6) { CLOB_V(60); CLOB_S(79); }   // 61 VGPRs + 80 SGPRs
  if (KIND == 7) { CLOB_V(60); CLOB_S(83); }   // 61 VGPRs + 84 SGPRs
  if (KIND == 8) { CLOB_V(60); CLOB_S(75); }   // 61 VGPRs + 76 SGPRs
  while (__builtin_amdgcn_s_memrealtime() - t0 < spin_ticks) __builtin_amdgcn_s_sleep(1);
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63u) == 0u) {
    uint32_t xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    rec[blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6)] = make_uint4((uint32_t)t0, (uint32_t)t1, xcc, hw);
  }
}

template <int KIND, int BLOCK = 128>
static void run(const char* what, int cus) {
  constexpr uint32_t WPB = BLOCK / 64;            // waves per workgroup
  const uint32_t blocks = (uint32_t)cus * 48u / WPB;  // more waves than any residency limit allows at once
  uint4* d = nullptr;
  (void)hipMalloc(&d, blocks * WPB * sizeof(uint4));
  (void)hipMemset(d, 0, blocks * WPB * sizeof(uint4));
  int nb = 0;
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(&k_probe<KIND, BLOCK>), BLOCK, 0);
  hipFuncAttributes fa{};
  (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&k_probe<KIND, BLOCK>));
  hipLaunchKernelGGL((k_probe<KIND, BLOCK>), dim3(blocks), dim3(BLOCK), 0, 0, d, 5000u);  // warm
  (void)hipDeviceSynchronize();
  hipLaunchKernelGGL((k_probe<KIND, BLOCK>), dim3(blocks), dim3(BLOCK), 0, 0, d, 5000u);  // 50 us per wave
  (void)hipDeviceSynchronize();
  std::vector<uint4> h(blocks * WPB);
  (void)hipMemcpy(h.data(), d, h.size() * sizeof(uint4), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  // per SIMD (XCC, SE, SH, CU, SIMD): the most waves resident at once (ends before starts at equal clocks)
  std::map<uint64_t, std::vector<std::pair<uint32_t, int>>> ev;
  uint32_t slot_max = 0;
  for (const uint4& r : h) {
    const uint64_t key = ((uint64_t)r.z << 16) | (((r.w >> 8) & 0xffu) << 4) | ((r.w >> 4) & 3u);
    ev[key].push_back({r.x, +1});
    ev[key].push_back({r.y, -1});
    slot_max = std::max(slot_max, r.w & 0xfu);
  }
  int best = 0;
  size_t at_best = 0;
  for (auto& kv : ev) {
    auto& v = kv.second;
    std::sort(v.begin(), v.end(), [](const std::pair<uint32_t, int>& a, const std::pair<uint32_t, int>& b) {
      return a.first != b.first ? a.first < b.first : a.second < b.second;
    });
    int cur = 0, m = 0;
    for (const auto& e : v) m = std::max(m, cur += e.second);
    if (m > best) {
      best = m;
      at_best = 0;
    }
    if (m == best) ++at_best;
  }
  std::printf("{\"kernel\": \"%s\", \"block\": %d, \"vgprs\": %d, \"runtime_blocks_per_cu\": %d, "
              "\"runtime_waves_per_simd\": %.2f, \"measured_max_waves_per_simd\": %d, \"simds_at_max\": %zu, "
              "\"simds\": %zu, \"hw_wave_slot_max\": %u}\n",
              what, BLOCK, fa.numRegs, nb, nb * (double)WPB / 4.0, best, at_best, ev.size(), slot_max);
}

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  run<0>("few registers", cus);
  run<1>("61 VGPRs", cus);
  run<2>("64 VGPRs", cus);
  run<3>("65 VGPRs", cus);
  run<4>("61 VGPRs + 88 SGPRs", cus);
  run<5>("100 SGPRs", cus);
  run<6>("61 VGPRs + 80 SGPRs", cus);
  run<7>("61 VGPRs + 84 SGPRs", cus);
  run<8>("61 VGPRs + 76 SGPRs", cus);
  run<0, 64>("few registers, 1-wave workgroups", cus);
  run<0, 256>("few registers, 4-wave workgroups", cus);
  run<1, 256>("61 VGPRs, 4-wave workgroups", cus);
  run<4, 256>("61 VGPRs + 88 SGPRs, 4-wave workgroups", cus);
  return 0;
}
