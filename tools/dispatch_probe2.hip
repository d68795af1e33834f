// dispatch_probe2.hip — why qf_fuse's empty sort launch costs twice the wave-launch
// rate that tools/dispatch_probe.hip measured (development).  Each variant is a
// 512-thread, 36 KB-LDS launch of 20,712 workgroups that all exit after reading their
// pair's union count, launched right after a "join" kernel that wrote those counts
// (one workgroup per query, as the join does); rocprofv3 --kernel-trace gives each
// kernel's duration.  Variants (template MODE):
//   0: the counts were written by the previous kernel; small kernel arguments
//   1: as 0, with a 256-byte by-value argument struct read in two dependent batches
//      (the sort kernels' FuseParams shape) and the 2-D grid's block id
//   2: as 1, but the previous kernel did not write the counts (they stay L2 / MALL-
//      resident from the launch before)
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ab/dispatch_probe2 tools/dispatch_probe2.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("%s\n", hipGetErrorString(err_)); return 1; } } while (0)

struct Args {  // FuseParams-like: 32 eight-byte fields
  int64_t n_queries;
  int32_t R, methods;
  const int64_t* list_off;
  int32_t* union_count;
  int64_t pad[28];
};

__global__ __launch_bounds__(512) void writer_k(int32_t* __restrict__ cnt, int n, int v) {
  // one workgroup per query, as the join: thread 0 writes its count
  if (threadIdx.x == 0 && (int)blockIdx.x < n) cnt[blockIdx.x] = v;
}

__global__ __launch_bounds__(512) void empty_small(const int32_t* __restrict__ cnt, int nq, int M,
                                                   int* __restrict__ out) {
  __shared__ int lds[36864 / 4];
  const int b = blockIdx.x;
  const int q = (b >> 3) / M * 8 + (b & 7);
  if (q >= nq) return;
  const int U = cnt[q];
  if (U <= 3072) {  // never taken here (counts are 4,000)
    lds[threadIdx.x] = U;
    __syncthreads();
    out[b] = lds[(threadIdx.x + 1) & 511];
  }
}

__global__ __launch_bounds__(512) void empty_params(Args p, int* __restrict__ out) {
  __shared__ int lds[36864 / 4];
  const int64_t bid = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
  const int M = __popc(p.methods);
  const int64_t grp8 = bid >> 3, ngroups = (p.n_queries + 7) / 8;
  if (grp8 >= ngroups * M) return;
  const int64_t q = (ngroups - 1 - grp8 / M) * 8 + (bid & 7);
  if (q >= p.n_queries) return;
  const int U = p.union_count[q];
  if (U <= 3072) {
    lds[threadIdx.x] = U + (int)p.pad[(int)(bid & 15)];
    __syncthreads();
    out[bid] = lds[(threadIdx.x + 1) & 511];
  }
}

// P: bsort_fast_kernel's prologue pieces on FuseParams-shaped arguments.
//   V1: 1-D block id, grp8 / M by a host magic (an argument), U, exit
//   V2: V1 with the magic computed in the kernel (0xFFFFFFFF / M + 1: a u32 division)
//   V3: V2 with the 2-D grid's block id (gridDim.x)
//   V4: V3 with the 64-bit division fallback for grp8 >= 2^20 in the code (not taken)
//   V5: V4 plus the learned-slot test and the list offsets loaded beside U (the
//       kernel's exact prologue)
template <int V>
__global__ __launch_bounds__(512) void empty_v(Args p, uint32_t magic, int* __restrict__ out) {
  __shared__ int lds[36864 / 4];
  const int64_t bid = V >= 3 ? (int64_t)blockIdx.y * gridDim.x + blockIdx.x : (int64_t)blockIdx.x;
  const int M = __popc(p.methods);
  const int64_t grp8 = bid >> 3, ngroups = (p.n_queries + 7) / 8;
  if (grp8 >= ngroups * M) return;
  const uint32_t mg = V >= 2 ? 0xFFFFFFFFu / (uint32_t)M + 1u : magic;
  int64_t gq;
  if (V >= 4) {
    if (M == 1) gq = grp8;
    else if (grp8 < (1 << 20)) gq = (int64_t)__umulhi((uint32_t)grp8, mg);
    else gq = grp8 / M;
  } else {
    gq = M == 1 ? grp8 : (int64_t)__umulhi((uint32_t)grp8, mg);
  }
  const int64_t q = (ngroups - 1 - gq) * 8 + (bid & 7);
  const int ms = (int)(grp8 - gq * M);
  if (V >= 5 && (p.methods & 64) && ms == __popc(p.methods & 63)) return;
  if (q >= p.n_queries) return;
  const int U = p.union_count[q];
  int64_t base = 0, nqe = 0;
  if (V >= 5) {
    base = p.list_off[q * p.R];
    nqe = p.list_off[q * p.R + p.R] - base;
  }
  if (U < 1 || U <= 3072 + (int)(nqe & 0) || U > 5120) return;  // (counts 4,000: taken
  // by none of these — every workgroup exits here, as the small configuration's on C2)
  lds[threadIdx.x] = U + (int)base;
  __syncthreads();
  out[bid] = lds[(threadIdx.x + 1) & 511];
}

int main() {
  const int nq = 3452, M = 6, grid = (nq + 7) / 8 * 8 * M;
  int32_t* cnt;
  int* out;
  CK(hipMalloc(&cnt, nq * sizeof(int32_t)));
  CK(hipMalloc(&out, (size_t)grid * sizeof(int)));
  Args a{};
  a.n_queries = nq;
  a.R = 5;
  a.methods = 63;
  a.union_count = cnt;
  int64_t* loff;
  CK(hipMalloc(&loff, (size_t)(nq * 5 + 1) * sizeof(int64_t)));
  CK(hipMemset(loff, 0, (size_t)(nq * 5 + 1) * sizeof(int64_t)));
  a.list_off = loff;
  for (int rep = 0; rep < 20; ++rep) {
    // 0: written by the previous kernel, small arguments
    hipLaunchKernelGGL(writer_k, dim3(nq), dim3(512), 0, 0, cnt, nq, 4000);
    hipLaunchKernelGGL(empty_small, dim3(grid), dim3(512), 0, 0, cnt, nq, M, out);
    // 1: written by the previous kernel, FuseParams-shaped arguments
    hipLaunchKernelGGL(writer_k, dim3(nq), dim3(512), 0, 0, cnt, nq, 4000);
    hipLaunchKernelGGL(empty_params, dim3(grid), dim3(512), 0, 0, a, out);
    // 2: not written just before
    hipLaunchKernelGGL(empty_params, dim3(grid), dim3(512), 0, 0, a, out);
    const uint32_t magic = 0xFFFFFFFFu / 6u + 1u;
    hipLaunchKernelGGL(writer_k, dim3(nq), dim3(512), 0, 0, cnt, nq, 4000);
    hipLaunchKernelGGL(empty_v<1>, dim3(grid), dim3(512), 0, 0, a, magic, out);
    hipLaunchKernelGGL(writer_k, dim3(nq), dim3(512), 0, 0, cnt, nq, 4000);
    hipLaunchKernelGGL(empty_v<2>, dim3(grid), dim3(512), 0, 0, a, magic, out);
    hipLaunchKernelGGL(writer_k, dim3(nq), dim3(512), 0, 0, cnt, nq, 4000);
    hipLaunchKernelGGL(empty_v<3>, dim3(grid), dim3(512), 0, 0, a, magic, out);
    hipLaunchKernelGGL(writer_k, dim3(nq), dim3(512), 0, 0, cnt, nq, 4000);
    hipLaunchKernelGGL(empty_v<4>, dim3(grid), dim3(512), 0, 0, a, magic, out);
    hipLaunchKernelGGL(writer_k, dim3(nq), dim3(512), 0, 0, cnt, nq, 4000);
    hipLaunchKernelGGL(empty_v<5>, dim3(grid), dim3(512), 0, 0, a, magic, out);
  }
  CK(hipDeviceSynchronize());
  printf("done %d workgroups per empty launch\n", grid);
  CK(hipFree(cnt));
  CK(hipFree(loff));
  CK(hipFree(out));
  return 0;
}
