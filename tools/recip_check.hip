// Exhaustive check (GPU): is a short Newton-refined reciprocal bit-equal to the IEEE quotient 1.0f / x (what the
// oracle computes on the CPU)? Every 32-bit pattern with exponent field in [lo, hi] (both signs) is tested:
//   A  v_rcp_f32 + one fused Newton step, unguarded (rcp_exact's fast path)
//   B  two Newton steps
//   E  rt::rcp_exact itself (rt_device.hpp: the fast path where the exponent is in [20, 234], the IEEE division
//      for the rest of the wave otherwise), the function the trace kernel's triangle test calls
// Prints the mismatch counts and the first mismatching patterns. Built by the Makefile (tools/bin/recip_check);
// tests/test_gpu_rcp.py runs it.
//   ./recip_check [lo_exp hi_exp]   (biased exponents; default 0 255: every float, zeros / denormals / inf / NaN
//   included; A and B are meaningful inside [20, 234] only)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../realtimeraytracing_gradproject_amd/csrc/rt_device.hpp"

__device__ __forceinline__ float ieee_recip(float x) {
  float r;
  // the compiler's correctly rounded division (div_scale / rcp / fma / div_fmas / div_fixup)
  r = 1.0f / x;
  return r;
}

// A: one Newton step with fused residual
__device__ __forceinline__ float recip_a(float x) {
  const float r = __builtin_amdgcn_rcpf(x);
  const float e = __builtin_fmaf(-x, r, 1.0f);
  return __builtin_fmaf(e, r, r);
}

// B: two steps
__device__ __forceinline__ float recip_b(float x) {
  const float r = recip_a(x);
  const float e = __builtin_fmaf(-x, r, 1.0f);
  return __builtin_fmaf(e, r, r);
}

__global__ void k_check(uint32_t lo_exp, uint32_t hi_exp, unsigned long long* bad, uint32_t* first) {
  // exhaustive over the range; every wave runs whole (the guarded rcp_exact ballots over the wave)
  const uint64_t n_per_sign = (uint64_t)(hi_exp - lo_exp + 1) << 23;
  const uint64_t total = n_per_sign * 2;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t j = i % n_per_sign;
    const uint32_t sign = i < n_per_sign ? 0u : 0x80000000u;
    const uint32_t bits = sign | ((lo_exp << 23) + (uint32_t)j);
    const float x = __uint_as_float(bits);
    const uint32_t ref = __float_as_uint(ieee_recip(x));
    const uint32_t a = __float_as_uint(recip_a(x));
    const uint32_t b = __float_as_uint(recip_b(x));
    if (a != ref) {
      const unsigned long long k = atomicAdd(&bad[0], 1ull);
      if (k < 8) first[k] = bits;
    }
    if (b != ref) {
      const unsigned long long k = atomicAdd(&bad[1], 1ull);
      if (k < 8) first[8 + k] = bits;
    }
    const float ef = rt::rcp_exact(x);
    const uint32_t e = __float_as_uint(ef);
    if (x != x ? ef == ef : e != ref) {  // NaN in: any NaN out
      const unsigned long long k = atomicAdd(&bad[2], 1ull);
      if (k < 8) first[16 + k] = bits;
    }
  }
}

int main(int argc, char** argv) {
  const uint32_t lo = argc > 2 ? (uint32_t)atoi(argv[1]) : 0u;
  const uint32_t hi = argc > 2 ? (uint32_t)atoi(argv[2]) : 255u;
  if (hi > 255 || lo > hi) return 2;
  unsigned long long* bad;
  uint32_t* first;
  if (hipMalloc(&bad, 24) != hipSuccess || hipMalloc(&first, 96) != hipSuccess) return 3;
  (void)hipMemset(bad, 0, 24);
  (void)hipMemset(first, 0, 96);
  hipLaunchKernelGGL(k_check, dim3(8192), dim3(256), 0, 0, lo, hi, bad, first);
  if (hipDeviceSynchronize() != hipSuccess) return 4;
  unsigned long long hb[3];
  uint32_t hf[24];
  (void)hipMemcpy(hb, bad, 24, hipMemcpyDeviceToHost);
  (void)hipMemcpy(hf, first, 96, hipMemcpyDeviceToHost);
  std::printf("exponents [%u, %u], both signs: %llu patterns\n", lo, hi, (unsigned long long)(hi - lo + 1) << 24);
  std::printf("A (rcp + 1 fma step): %llu mismatches", hb[0]);
  for (int k = 0; k < 8 && k < (int)hb[0]; ++k) std::printf(" %08x", hf[k]);
  std::printf("\nB (rcp + 2 fma steps): %llu mismatches", hb[1]);
  for (int k = 0; k < 8 && k < (int)hb[1]; ++k) std::printf(" %08x", hf[8 + k]);
  std::printf("\nE (rt::rcp_exact, guarded): %llu mismatches", hb[2]);
  for (int k = 0; k < 8 && k < (int)hb[2]; ++k) std::printf(" %08x", hf[16 + k]);
  std::printf("\n");
  return 0;
}
