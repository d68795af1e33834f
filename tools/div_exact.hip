// Probe (development): the division-free quotients of the join kernel against
// IEEE division, bit for bit, on the GPU itself.
//   micro:  m / 1e6 for every int32 m        (qf_common.h micro_to_f64)
//   recip:  1 / n for every n in [1, 2^24]   (qf_common.h recip_small)
//   quot:   w / n for 2^32 pseudo-random (w, n), w of every magnitude, n <= 2^24
//           (qf_common.h div_small)
//   unit:   a / b for 2^32 pseudo-random doubles b of every magnitude and a in [0, b]
//           with y = 1 / b computed once (qf_common.h div_by_recip: min-max scaling)
// Prints the mismatch count of each; the library relies on all four being 0.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../qpp-fusion-rag_amd/csrc/qf_common.h"

__device__ unsigned long long g_bad[4];

__global__ void micro(long long base) {
  const long long m = base + (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int32_t v = (int32_t)(uint32_t)m;
  const double want = (double)v / 1e6;
  const double got = qf::micro_to_f64(v);
  if (__double_as_longlong(want) != __double_as_longlong(got)) atomicAdd(&g_bad[0], 1ull);
}

__global__ void recip(int base) {
  const int n = base + blockIdx.x * blockDim.x + threadIdx.x;
  if (n < 1 || n > (1 << 24)) return;
  const double want = 1.0 / (double)n;
  if (__double_as_longlong(want) != __double_as_longlong(qf::recip_small(n)))
    atomicAdd(&g_bad[1], 1ull);
}

__global__ void quot(unsigned seed) {
  uint64_t h = ((uint64_t)seed << 32) ^ ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x);
  h ^= h >> 33; h *= 0xff51afd7ed558ccdull; h ^= h >> 33; h *= 0xc4ceb9fe1a85ec53ull; h ^= h >> 33;
  // w: random mantissa and sign, exponent in [-300, 300]; n: log-uniform in [1, 2^24]
  const int ex = (int)((h >> 52) % 601) - 300;
  const double w = ldexp(1.0 + (double)(h & ((1ull << 52) - 1)) * 0x1p-52, ex) * ((h >> 63) ? -1.0 : 1.0);
  uint64_t g = h * 0x9E3779B97F4A7C15ull;
  g ^= g >> 29;
  const int nb = (int)(g % 24);
  const int n = (int)(((g >> 8) & ((1u << nb) - 1)) | (1u << nb));
  const double want = w / (double)n;
  if (__double_as_longlong(want) != __double_as_longlong(qf::div_small(w, n)))
    atomicAdd(&g_bad[2], 1ull);
}

__global__ void unit(unsigned seed) {
  uint64_t h = ((uint64_t)seed << 32) ^ ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x);
  h ^= h >> 33; h *= 0xff51afd7ed558ccdull; h ^= h >> 33; h *= 0xc4ceb9fe1a85ec53ull; h ^= h >> 33;
  const int ex = (int)((h >> 52) % 1601) - 800;
  const double b = ldexp(1.0 + (double)(h & ((1ull << 52) - 1)) * 0x1p-52, ex);
  uint64_t g = h * 0x9E3779B97F4A7C15ull;
  g ^= g >> 31; g *= 0xbf58476d1ce4e5b9ull; g ^= g >> 29;
  // a = b * t, t in (0, 1]: uniform mantissa, and every 4th a tiny fraction of b
  double t = (double)((g >> 11) | 1) * 0x1p-53;
  if ((g & 3) == 0) t = ldexp(t, -(int)((g >> 2) % 60));
  const double a = b * t;
  const double y = 1.0 / b;
  if (!(a >= 0x1p-900)) return;  // the fast path's domain
  const double want = a / b;
  if (__double_as_longlong(want) != __double_as_longlong(qf::div_by_recip(a, b, y)))
    atomicAdd(&g_bad[3], 1ull);
}

int main() {
  unsigned long long zero[4] = {0, 0, 0, 0}, bad[4];
  hipMemcpyToSymbol(HIP_SYMBOL(g_bad), zero, sizeof zero);
  for (long long b = 0; b < (1ll << 32); b += (1ll << 30))
    hipLaunchKernelGGL(micro, dim3(1 << 22), dim3(256), 0, 0, b);
  hipLaunchKernelGGL(recip, dim3((1 << 24) / 256 + 1), dim3(256), 0, 0, 0);
  for (unsigned s = 0; s < 16; ++s) hipLaunchKernelGGL(quot, dim3(1 << 20), dim3(256), 0, 0, s);
  for (unsigned s = 0; s < 16; ++s) hipLaunchKernelGGL(unit, dim3(1 << 20), dim3(256), 0, 0, s);
  hipDeviceSynchronize();
  hipMemcpyFromSymbol(bad, HIP_SYMBOL(g_bad), sizeof bad);
  printf("{\"micro_all_int32\": %llu, \"recip_1_to_2^24\": %llu, \"quot_2^32_random\": %llu, "
         "\"unit_2^32_random\": %llu}\n", bad[0], bad[1], bad[2], bad[3]);
  return (bad[0] | bad[1] | bad[2] | bad[3]) ? 1 : 0;
}
