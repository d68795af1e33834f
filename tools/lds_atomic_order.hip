// Probe (development): are same-address LDS atomics of one wave instruction
// applied in lane order on gfx950?  Each lane atomically increments the counter
// of its digit and compares the returned value with the number of lower lanes
// holding the same digit.  Prints the violation count over many random rows.
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ unsigned g_bad;
__global__ __launch_bounds__(512) void probe(int trials, int bits, unsigned seed) {
  __shared__ unsigned cnt[8][512];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  unsigned bad = 0;
  for (int t = 0; t < trials; ++t) {
    for (int k = lane; k < 512; k += 64) cnt[wid][k] = 0;
    __syncthreads();
    unsigned h = seed ^ (blockIdx.x * 0x9E3779B9u) ^ (t * 0x85EBCA6Bu) ^ (threadIdx.x * 0xC2B2AE35u);
    h ^= h >> 16; h *= 0x7FEB352Du; h ^= h >> 15; h *= 0x846CA68Bu; h ^= h >> 16;
    const unsigned mode = (t >> 4) & 3;
    unsigned d = h & ((1u << bits) - 1);
    if (mode == 1) d &= 3;          // few distinct digits: long same-address runs
    if (mode == 2) d = 7;           // every lane the same address
    if (mode == 3) d = (lane * 37 + t) & ((1u << bits) - 1);
    const unsigned r = atomicAdd(&cnt[wid][d], 1u);
    // expected: lanes below me with the same digit
    unsigned before = 0;
    for (int l = 0; l < 64; ++l) {
      const unsigned dl = __shfl(d, l, 64);
      if (l < lane && dl == d) ++before;
    }
    bad += (r != before);
    __syncthreads();
  }
  if (bad) atomicAdd(&g_bad, bad);
}
int main() {
  unsigned zero = 0, bad = 0;
  hipMemcpyToSymbol(HIP_SYMBOL(g_bad), &zero, sizeof zero);
  for (int bits = 1; bits <= 9; bits += 4)
    hipLaunchKernelGGL(probe, dim3(2048), dim3(512), 0, 0, 256, bits, 12345u + bits);
  hipDeviceSynchronize();
  hipMemcpyFromSymbol(&bad, HIP_SYMBOL(g_bad), sizeof bad);
  printf("{\"rows_checked\": %lld, \"violations\": %u}\n", 3LL * 2048 * 8 * 256, bad);
  return 0;
}
