// copy_probe.hip — which streaming-copy shape reaches the HBM copy ceiling on
// MI355X (the roofline's measured ceiling: qf_stream_copy in csrc/qf_norm.hip).
// Variants: non-temporal or plain 16-byte accesses, 1/2/4/8 accesses in flight
// per lane, grid sizes.  Prints GB/s (read + write bytes / time) per variant.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/copy_probe tools/copy_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_k(u32x4* __restrict__ d, const u32x4* __restrict__ s,
                                              long n) {
  const long stride = (long)gridDim.x * 256;
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = NT ? __builtin_nontemporal_load(&s[i + k * stride]) : s[i + k * stride];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (NT) __builtin_nontemporal_store(v[k], &d[i + k * stride]);
      else d[i + k * stride] = v[k];
    }
  }
  for (; i < n; i += stride) d[i] = s[i];
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int U, bool NT>
int run(u32x4* d, u32x4* s, long n, int blocks, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL((copy_k<U, NT>), dim3(blocks), dim3(256), 0, 0, d, s, n);
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((copy_k<U, NT>), dim3(blocks), dim3(256), 0, 0, d, s, n);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  printf("{\"unroll\": %d, \"nt\": %d, \"blocks\": %d, \"bytes\": %ld, \"gbs\": %.1f}\n", U, (int)NT,
         blocks, n * 16, 2.0 * n * 16 / (ms / reps * 1e-3) / 1e9);
  return 0;
}

int main(int argc, char** argv) {
  const long bytes = argc > 1 ? atol(argv[1]) : (1L << 30);
  const long n = bytes / 16;
  u32x4 *s, *d;
  CK(hipMalloc(&s, bytes));
  CK(hipMalloc(&d, bytes));
  CK(hipMemset(s, 1, bytes));
  CK(hipMemset(d, 0, bytes));
  const int reps = 20;
  if (argc > 2) {  // round 4: fewer workgroups per CU, and the one-shot grid (one access per thread)
    for (int blocks : {256, 512, 768, 1024, 1280, (int)((n + 255) / 256)}) {
      run<1, false>(d, s, n, blocks, reps);
      run<1, true>(d, s, n, blocks, reps);
      run<2, true>(d, s, n, blocks, reps);
    }
  } else {
    for (int blocks : {1024, 2048, 4096}) {
      run<1, false>(d, s, n, blocks, reps);
      run<4, false>(d, s, n, blocks, reps);
      run<8, false>(d, s, n, blocks, reps);
      run<1, true>(d, s, n, blocks, reps);
      run<4, true>(d, s, n, blocks, reps);
      run<8, true>(d, s, n, blocks, reps);
    }
  }
  CK(hipFree(s));
  CK(hipFree(d));
  return 0;
}
