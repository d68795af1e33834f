// qf_lists.h — per-list device bodies shared by kernels in different files (the
// library is built without relocatable device code): the per-query min-max of
// normalize_scores and the QPP column min / max.
#pragma once

#include "qf_common.h"

namespace qf {

// normalize_scores of one list held in registers: ROWS rows of 64 entries (every
// load in flight before the first use, the rows past the list masked).
template <int ROWS>
__device__ __forceinline__ void minmax_list_rows(const double* __restrict__ score, int64_t a,
                                                 int64_t b, double* __restrict__ out_norm,
                                                 int32_t* __restrict__ out_micro) {
  const int lane = threadIdx.x & 63;
  double v[ROWS];
  double mn = INFINITY, mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < ROWS; ++j) {  // every load in flight before the first use
    const int64_t i = a + j * 64 + lane;
    v[j] = i < b ? score[i] : 0.0;  // (non-temporal: 39.5 -> 41.6 us, not kept)
  }
#pragma unroll
  for (int j = 0; j < ROWS; ++j)
    if (a + j * 64 + lane < b) {
      mn = fmin(mn, v[j]);
      mx = fmax(mx, v[j]);
    }
  mn = wave_min(mn);
  mx = wave_max(mx);
  const double range = mx > mn ? mx - mn : 1.0;
  const double y = 1.0 / range;  // one IEEE division per list
  const bool fast = range >= 0x1p-900 && range <= 0x1p900;
#pragma unroll
  for (int j = 0; j < ROWS; ++j) {
    const int64_t i = a + j * 64 + lane;
    if (i < b) {
      const double d = v[j] - mn;
      const double x = (fast && d >= 0x1p-900 && d <= 0x1p900) ? div_by_recip(d, range, y)
                                                               : d / range;
      if (out_norm) out_norm[i] = x;
      if (out_micro) out_micro[i] = (int32_t)round6(x);
    }
  }
}

// normalize_scores (src/retrievers/base.py:60-73) of list l, one wavefront.
__device__ __forceinline__ void minmax_list(const double* __restrict__ score,
                                            const int64_t* __restrict__ list_off, int64_t l,
                                            double* __restrict__ out_norm,
                                            int32_t* __restrict__ out_micro) {
  const int lane = threadIdx.x & 63;
  const int64_t a = list_off[l], b = list_off[l + 1];
  // lists of <= 1024 entries: one HBM read, held in registers; up to 256 (C1's top-100)
  // in 4 rows, not 16 masked ones (C1's min-max 10.8 -> 9.4 us; a uniform row test in
  // the 16-row form instead cost top-1000 lists 2.5 us)
  if (b - a <= 256) {
    minmax_list_rows<4>(score, a, b, out_norm, out_micro);
    return;
  }
  if (b - a <= 1024) {
    minmax_list_rows<16>(score, a, b, out_norm, out_micro);
    return;
  }
  double mn = INFINITY, mx = -INFINITY;
  for (int64_t i = a + lane; i < b; i += 64) {
    const double s = score[i];
    mn = fmin(mn, s);
    mx = fmax(mx, s);
  }
  mn = wave_min(mn);
  mx = wave_max(mx);
  const double range = mx > mn ? mx - mn : 1.0;
  const double y = 1.0 / range;
  const bool fast = range >= 0x1p-900 && range <= 0x1p900;
  for (int64_t i = a + lane; i < b; i += 64) {
    const double d = score[i] - mn;
    const double v = (fast && d >= 0x1p-900 && d <= 0x1p900) ? div_by_recip(d, range, y)
                                                             : d / range;
    if (out_norm) out_norm[i] = v;
    if (out_micro) out_micro[i] = (int32_t)round6(v);
  }
}


// Column min / -max over present queries; one workgroup per (retriever, column).
__device__ __forceinline__ void qpp_colminmax_block(const double* __restrict__ raw,
                                                    const int64_t* __restrict__ list_off,
                                                    int64_t Q, int32_t R, double* __restrict__ mm,
                                                    int rc) {  // rc = r * 13 + c; 256 threads
  __shared__ double smin[4], smax[4];
  const int r = rc / kQppCols, c = rc % kQppCols;
  double vmin = INFINITY, vmax = -INFINITY;
  // 8 queries per thread per step, their loads in flight together
  constexpr int kU = 8;
  for (int64_t q0 = threadIdx.x; q0 < Q; q0 += (int64_t)blockDim.x * kU) {
    double v[kU];
    bool pr[kU];
#pragma unroll
    for (int t = 0; t < kU; ++t) {
      const int64_t q = q0 + (int64_t)t * blockDim.x;
      const int64_t l = q * R + r;
      pr[t] = q < Q && list_off[l + 1] > list_off[l];
      v[t] = q < Q ? raw[l * kQppCols + c] : 0.0;
    }
#pragma unroll
    for (int t = 0; t < kU; ++t)
      if (pr[t]) {
        vmin = fmin(vmin, v[t]);
        vmax = fmax(vmax, v[t]);
      }
  }
  vmin = wave_min(vmin);
  vmax = wave_max(vmax);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { smin[wid] = vmin; smax[wid] = vmax; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x / 64); ++w) {
      vmin = fmin(vmin, smin[w]);
      vmax = fmax(vmax, smax[w]);
    }
    mm[rc] = vmin;
    mm[R * kQppCols + rc] = -vmax;
  }
}

// One raw QPP value normalised as src/qpp.py:356-372 does — mode 1 (minmax: m0 =
// the column min, m1 = minus its max), 2 (zscore: m0 = mean, m1 = scale), 0 (none)
// — and 0.0 for a query whose list is absent (src/qpp.py:321).
__device__ __forceinline__ double qpp_norm_value(double x, double m0, double m1, int mode,
                                                 bool present) {
  double v = x;
  if (mode == 1) {
    const double vmin = m0;
    const double vmax = -m1;
    const double scale = vmax > vmin ? vmax - vmin : 1.0;
    v = scale > 0.0 ? (x - vmin) / scale : 0.0;
  } else if (mode == 2) {  // zscore: mm = [mean, scale] (qpp_colmeanstd)
    v = (x - m0) / m1;
  }
  return present ? v : 0.0;
}
// float("%.6f") of the written text: m / 1e6 (division-free where checked exact).
__device__ __forceinline__ double micro_back(long long m) {
  return (m > -0x7FFFFFFFll && m < 0x7FFFFFFFll) ? micro_to_f64((int32_t)m) : (double)m / 1e6;
}

}  // namespace qf
