// VALU issue-rate probe (development): 32-bit integer ops per SIMD-cycle at full
// occupancy, to price the sort kernel's VALU rate.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(256) void valu_kernel(unsigned* out, int iters) {
  unsigned a = threadIdx.x, b = a * 3 + 1, c = a ^ 0x55, d = a + 7, e = a * 5, f = a ^ 0x99,
           g = a + 11, h = a * 13;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {  // 8 independent chains x 16 = 128 VALU per iteration
      a = (a ^ b) + 0x9E37u; b = (b ^ c) + 0x79B9u; c = (c ^ d) + 0x7F4Au; d = (d ^ e) + 0x7C15u;
      e = (e ^ f) + 0x1234u; f = (f ^ g) + 0x5678u; g = (g ^ h) + 0x9ABCu; h = (h ^ a) + 0xDEF0u;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;
}
int main() {
  unsigned* out;
  const int blocks = 256 * 32, threads = 256, iters = 200;  // 8 waves per SIMD
  hipMalloc(&out, sizeof(unsigned) * blocks * threads);
  hipLaunchKernelGGL(valu_kernel, dim3(blocks), dim3(threads), 0, 0, out, 10);
  hipDeviceSynchronize();
  hipEvent_t t0, t1;
  hipEventCreate(&t0);
  hipEventCreate(&t1);
  hipEventRecord(t0);
  hipLaunchKernelGGL(valu_kernel, dim3(blocks), dim3(threads), 0, 0, out, iters);
  hipEventRecord(t1);
  hipEventSynchronize(t1);
  float ms;
  hipEventElapsedTime(&ms, t0, t1);
  const double waves = (double)blocks * threads / 64, instr = waves * iters * 16 * 8;  // v_xad_u32 each
  printf("{\"ms\": %.4f, \"wave_valu_instr\": %.3e, \"instr_per_simd_per_ns\": %.4f}\n", ms, instr,
         instr / 1024 / (ms * 1e6));
  return 0;
}
