// qf_norm.hip — per-query min-max normalisation of run lists (.res -> .norm.res)
// and the on-device synthetic run generator used by bench.py / the GPU tests.
//
// normalize_scores (src/retrievers/base.py:60-73), applied by write_run before
// "%.6f" (scripts/02_retrieve.py:76-80): one wavefront per list, wave min/max
// reduction, then (s - min) / range with range = 1.0 when max == min.
#include "qf_common.h"
#include "qf_internal.h"
#include "qf_lists.h"

namespace qf {

__global__ __launch_bounds__(256) void minmax_per_query_kernel(
    const double* __restrict__ score, const int64_t* __restrict__ list_off, int64_t n_lists,
    double* __restrict__ out_norm, int32_t* __restrict__ out_micro) {
  const int64_t l = block_id() * 4 + (threadIdx.x >> 6);
  if (l >= n_lists) return;
  minmax_list(score, list_off, l, out_norm, out_micro);
}

// The unsharded step's two independent reductions in one launch: the QPP column
// min / max workgroups first (latency-bound, R * 13 of them), then the per-list
// min-max ones — the column pass runs beside the streaming one instead of as a
// launch of its own (qf_minmax_colminmax; the same bits as the two kernels).
__global__ __launch_bounds__(256) void minmax_colminmax_kernel(
    const double* __restrict__ score, const int64_t* __restrict__ list_off, int64_t Q, int32_t R,
    double* __restrict__ out_norm, int32_t* __restrict__ out_micro,
    const double* __restrict__ raw, double* __restrict__ mm) {
  const int64_t bid = block_id(), ncol = (int64_t)R * kQppCols;
  if (bid < ncol) {
    qpp_colminmax_block(raw, list_off, Q, R, mm, (int)bid);
    return;
  }
  const int64_t l = (bid - ncol) * 4 + (threadIdx.x >> 6);
  if (l >= Q * R) return;
  minmax_list(score, list_off, l, out_norm, out_micro);
}

hipError_t minmax_launch(const double* score, const int64_t* list_off, int64_t n_lists,
                         double* out_norm, int32_t* out_micro, hipStream_t st) {
  if (n_lists == 0) return hipSuccess;
  hipLaunchKernelGGL(minmax_per_query_kernel, grid_for((n_lists + 3) / 4), dim3(256), 0,
                     st, score, list_off, n_lists, out_norm, out_micro);
  return hipGetLastError();
}

hipError_t minmax_colminmax_launch(const double* score, const int64_t* list_off, int64_t Q,
                                   int32_t R, double* out_norm, int32_t* out_micro,
                                   const double* raw, double* mm, hipStream_t st) {
  if (Q * R == 0) return hipSuccess;
  const int64_t blocks = (int64_t)R * kQppCols + (Q * R + 3) / 4;
  hipLaunchKernelGGL(minmax_colminmax_kernel, grid_for(blocks), dim3(256), 0, st, score, list_off,
                     Q, R, out_norm, out_micro, raw, mm);
  return hipGetLastError();
}

// ---- synthetic runs -----------------------------------------------------------
// Counter-based: every value is a pure function of (seed, global q, r, i), so any
// query range (a rank's shard) can be generated independently and re-generated.

__device__ __forceinline__ uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t hash4(uint64_t seed, uint64_t a, uint64_t b, uint64_t c) {
  return mix64(seed ^ mix64(a ^ mix64(b ^ mix64(c))));
}
__device__ __forceinline__ double u01(uint64_t h) { return (double)(h >> 11) * 0x1.0p-53; }

struct RetrieverProfile { double A, B, c; };
// BGE, BM25, BM25_MonoT5, BM25_TCT, Splade (sorted names, pickle order) and extras.
__constant__ RetrieverProfile kProfiles[8] = {
    {0.50, 0.40, 2.0},  {5.0, 25.0, 4.0},  {-12.0, 11.5, 3.0}, {60.0, 20.0, 2.5},
    {8.0, 30.0, 3.5},   {1.0, 2.0, 3.0},   {0.0, 1.0, 2.0},    {-1.0, 3.0, 3.0}};

__global__ __launch_bounds__(256) void synth_kernel(int64_t q_begin, int64_t n_queries, int32_t R,
                                                     int32_t K, uint64_t seed, double p_shared,
                                                     int64_t* __restrict__ list_off,
                                                     uint32_t* __restrict__ docid,
                                                     double* __restrict__ score) {
  const int64_t idx = block_id() * blockDim.x + threadIdx.x;
  const int64_t total = n_queries * R * (int64_t)K;
  if (idx == 0) list_off[n_queries * R] = total;
  if (idx >= total) return;
  const int i = (int)(idx % K);
  const int64_t lq = idx / K;  // local list index
  const int r = (int)(lq % R);
  const int64_t qg = q_begin + lq / R;  // global query index
  if (i == 0) list_off[lq] = lq * K;
  const int P = K;  // per-query shared candidate pool
  const uint64_t hl = hash4(seed, (uint64_t)qg, (uint64_t)r, 0xA11CEull);
  const uint64_t he = hash4(seed, (uint64_t)qg, (uint64_t)r, (uint64_t)i + 1);
  uint32_t d;
  if (u01(he) < p_shared) {
    // affine bijection of positions onto the pool: distinct within the list
    uint32_t A = (uint32_t)(hl % (uint64_t)P) | 1u;
    while (A > 1) {  // make A coprime with P
      uint32_t x = A, y = (uint32_t)P;
      while (y) { const uint32_t t = x % y; x = y; y = t; }
      if (x == 1) break;
      A += 2;
      if (A >= (uint32_t)P) A = 1;
    }
    // with probability 1/2 the list's first position maps to pool index 0..2 —
    // the documents the bench's synthetic qrels judge relevant
    const uint32_t B = ((hl >> 20) & 1u) ? (uint32_t)((hl >> 32) % 3u)
                                         : (uint32_t)((hl >> 32) % (uint64_t)P);
    const uint32_t pidx = (uint32_t)(((uint64_t)A * (uint64_t)i + B) % (uint64_t)P);
    d = (uint32_t)(((uint64_t)qg * (uint64_t)P + pidx) & 0x7FFFFFFFull);
  } else {
    const uint64_t hq = hash4(seed, (uint64_t)qg, 0xD0Cull, 0);
    // distinct within the query for r*K + i < 2^31 - 1; never 0xFFFFFFFF (reserved)
    d = 0x80000000u | (uint32_t)((hq + (uint64_t)r * (uint64_t)K + (uint64_t)i) % 0x7FFFFFFFull);
  }
  const RetrieverProfile pr = kProfiles[r & 7];
  const double jitter = 0.8 + 0.4 * u01(hash4(seed, (uint64_t)qg, (uint64_t)r, 0x5CA1Eull));
  const double t = ((double)i + 0.5 * u01(mix64(he))) / (double)K;
  const double s = pr.A + pr.B * jitter * exp(-pr.c * t);
  docid[idx] = d;
  score[idx] = s;
}

hipError_t synth_launch(int64_t q_begin, int64_t n_queries, int32_t R, int32_t K, uint64_t seed,
                        double p_shared, int64_t* list_off, uint32_t* docid, double* score,
                        hipStream_t st) {
  const int64_t total = n_queries * R * (int64_t)K;
  const int64_t blocks = total > 0 ? (total + 255) / 256 : 1;
  hipLaunchKernelGGL(synth_kernel, grid_for(blocks), dim3(256), 0, st, q_begin, n_queries, R,
                     K, seed, p_shared, list_off, docid, score);
  return hipGetLastError();
}

// ---- the HBM copy ceiling (measurement support) ------------------------------------
// A streaming copy, 16 bytes per lane, non-temporal, ONE access per thread over a
// one-shot grid (n16 / 256 workgroups): the practical read + write rate of HBM the
// roofline's achieved bytes are compared with.  tools/copy_probe.hip measured the
// shapes on MI355X (1 GiB): this one 6.57 TB/s (plain accesses 6.21); grid-stride
// loops over 1-5 workgroups per CU 3.2-5.9 TB/s, 2 / 4 / 8 accesses per lane in
// flight 4.3-5.8 (profiles/r04_copy_probe.jsonl, r04_copy_probe2.jsonl).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void stream_copy_kernel(u32x4* __restrict__ dst,
                                                          const u32x4* __restrict__ src,
                                                          int64_t n16) {
  const int64_t i = block_id() * 256 + threadIdx.x;
  if (i < n16) __builtin_nontemporal_store(__builtin_nontemporal_load(&src[i]), &dst[i]);
}

hipError_t stream_copy_launch(void* dst, const void* src, int64_t n16, hipStream_t st) {
  if (n16 <= 0) return hipSuccess;
  hipLaunchKernelGGL(stream_copy_kernel, grid_for((n16 + 255) / 256), dim3(256), 0, st,
                     (u32x4*)dst, (const u32x4*)src, n16);
  return hipGetLastError();
}

}  // namespace qf
