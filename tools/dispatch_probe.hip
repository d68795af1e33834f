// dispatch_probe.hip — what a launch of workgroups that all exit at once costs on
// MI355X (the empty sort configuration of qf_fuse's default path: DESIGN §8 "empty
// dispatch").  Variants: block size, static LDS per workgroup (which sets how many
// workgroups a CU holds), grid size, and what a workgroup does before it exits:
//   mode 0: nothing (no memory access),
//   mode 1: one load of its pair's flag (the sort kernels' union_count read),
//   mode 2: two dependent loads,
//   mode 3: four independent loads (one workgroup checking four pairs).
// Prints us per launch (hipEvents around 50 back-to-back launches; the floor is the
// 1-workgroup launch).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ab/dispatch_probe tools/dispatch_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("%s\n", hipGetErrorString(err_)); return 1; } } while (0)

template <int BLOCK, int LDSB, int MODE>
__global__ __launch_bounds__(BLOCK) void empty_k(const int* __restrict__ flag, int* __restrict__ out, int n) {
  __shared__ int lds[LDSB / 4];
  const int b = blockIdx.x;
  int v = 0;
  if (MODE == 1) v = flag[b];
  if (MODE == 2) v = flag[flag[b] + b];
  if (MODE == 3) v = flag[4 * b] | flag[4 * b + 1] | flag[4 * b + 2] | flag[4 * b + 3];
  if (MODE == 0) v = n < 0;  // never: keeps the LDS allocated
  if (v == 0) return;
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  out[b * BLOCK + threadIdx.x] = lds[(threadIdx.x + 1) % BLOCK];
}

template <int BLOCK, int LDSB, int MODE>
int run(const int* flag, int* out, int grid) {
  hipEvent_t a, e;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&e));
  const int reps = 50;
  hipLaunchKernelGGL((empty_k<BLOCK, LDSB, MODE>), dim3(grid), dim3(BLOCK), 0, 0, flag, out, grid);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((empty_k<BLOCK, LDSB, MODE>), dim3(grid), dim3(BLOCK), 0, 0, flag, out, grid);
  CK(hipEventRecord(e, 0));
  CK(hipEventSynchronize(e));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, e));
  printf("{\"block\": %d, \"lds\": %d, \"mode\": %d, \"grid\": %d, \"us\": %.2f}\n", BLOCK, LDSB, MODE,
         grid, ms * 1e3f / reps);
  return 0;
}

template <int BLOCK, int LDSB>
int sweep(const int* flag, int* out) {
  int rc = 0;
  for (int grid : {1, 2589, 5178, 10356, 20712, 41424}) {
    rc |= run<BLOCK, LDSB, 0>(flag, out, grid);
    rc |= run<BLOCK, LDSB, 1>(flag, out, grid);
    rc |= run<BLOCK, LDSB, 2>(flag, out, grid);
    if (grid <= 10356) rc |= run<BLOCK, LDSB, 3>(flag, out, grid);
  }
  return rc;
}

int main() {
  int *flag, *out;
  const int n = 4 * 41424;
  CK(hipMalloc(&flag, n * sizeof(int)));
  CK(hipMalloc(&out, (size_t)41424 * 1024 * sizeof(int)));  // (never written: flags 0)
  CK(hipMemset(flag, 0, n * sizeof(int)));
  int rc = 0;
  rc |= sweep<512, 4096>(flag, out);
  rc |= sweep<512, 36864>(flag, out);
  rc |= sweep<1024, 4096>(flag, out);
  rc |= sweep<1024, 73728>(flag, out);
  rc |= sweep<256, 4096>(flag, out);
  rc |= sweep<64, 4096>(flag, out);
  CK(hipFree(flag));
  CK(hipFree(out));
  return rc;
}
