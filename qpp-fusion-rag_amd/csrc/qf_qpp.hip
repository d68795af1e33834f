// qf_qpp.hip — score-distribution QPP predictors, one wavefront per list (gfx950).
//
// Replaces QPPBridge.computeQPPScores (src/qpp/java/qpp/QPPBridge.java:134-191)
// — formerly a JVM subprocess fed JSON (src/qpp.py:117-171) — and the driver's
// per-column min-max normalisation (src/qpp.py:340-374) + "%.6f" write-back
// (src/qpp.py:329-334) + get_qpp_weight (src/fusion.py:116-158).
//
// k = min(50, n) <= 64 values per list, so lane i holds rsv[i].  Java's
// sequential summation order is reproduced exactly: every sum that Java forms
// left-to-right is formed left-to-right here too (broadcast reads of rsv[j]
// from LDS, j uniform), and every DoubleStream.average() is the JDK's
// compensated (Kahan) sum.  Prefix statistics (SigmaMax, CumNQC) are lane
// parallel: lane i owns prefix rsv[0..i].
#include "qf_common.h"
#include "qf_internal.h"

namespace qf {

constexpr int kQppBlock = 256;  // 4 lists per workgroup

// v of lane l (l wave-uniform) as a scalar: two v_readlane_b32.
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// Java's left-to-right sum of t[0..k) (t held one per lane): a serial chain of
// scalar-broadcast adds, exactly the reference's order.
__device__ __forceinline__ double ordered_sum(double t, int k) {
  double acc = 0.0;
  for (int j = 0; j < k; ++j) acc += readlane_f64(t, j);
  return acc;
}

__global__ __launch_bounds__(kQppBlock) void qpp_raw_kernel(
    const double* __restrict__ score, const int64_t* __restrict__ list_off, int64_t n_lists,
    int32_t R, int32_t top_k, const int32_t* __restrict__ num_terms,
    const double* __restrict__ text_feat, double* __restrict__ out) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t l = (int64_t)blockIdx.x * (kQppBlock / 64) + wid;
  if (l >= n_lists) return;  // wave-uniform; no block barrier below
  const int64_t a = list_off[l], b = list_off[l + 1];
  int64_t n64 = b - a;
  if (top_k > 0 && n64 > top_k) n64 = top_k;  // sorted(...)[:top_k], src/qpp.py:305
  const int n = (int)n64;
  const int k = n < 50 ? n : 50;                 // QPPBridge.java:141
  double* o = out + l * kQppCols;
  if (k == 0) {  // empty map -> every column 0.0 (src/qpp.py:321)
    if (lane < kQppCols) o[lane] = 0.0;
    return;
  }
  const int64_t q = l / R;
  const bool act = lane < k;
  // float32 rounding of the JSON value (Gson getAsFloat), then widened.
  const double x = act ? (double)(float)score[a + lane] : 0.0;
  const int nt_raw = num_terms[q];
  const int numTerms = nt_raw > 1 ? nt_raw : 1;  // Math.max(1, terms.length)

  // prefix Kahan means (DoubleStream.average): lane i -> mean of rsv[0..i]
  Kahan kp;
  kahan_init(kp);
  for (int j = 0; j < k; ++j) {
    const double xj = readlane_f64(x, j);
    if (j <= lane) kahan_add(kp, xj);
  }
  const double mean_i = kahan_final(kp) / (double)(lane + 1);
  const double mu = readlane_f64(mean_i, k - 1);  // Arrays.stream(rsvs).average()

  // squared deviations around each prefix mean: simple sum -> NQC of the prefix
  // (NQC, CumNQC), compensated average -> population variance (SigmaMax, RSD)
  Kahan kv;
  kahan_init(kv);
  double sq = 0.0;
  for (int j = 0; j < k; ++j) {
    const double del = readlane_f64(x, j) - mean_i;
    const double d2 = del * del;  // Math.pow(s - mean, 2) == s*s exactly
    if (j <= lane) {
      sq += d2;
      kahan_add(kv, d2);
    }
  }
  const double nqc_i = sq / (double)(lane + 1);
  const double var_i = kahan_final(kv) / (double)(lane + 1);
  const double sigma_i = sqrt(var_i);
  const double nqc = readlane_f64(nqc_i, k - 1);          // col 0: NQC (:202-216)
  const double var_full = readlane_f64(var_i, k - 1);
  double sm = (lane >= 1 && act) ? sigma_i : 0.0;          // col 3: SigmaMax (:269-293)
  sm = wave_max(sm);
  const double sigmamax = k < 2 ? 0.0 : sm / sqrt((double)numTerms);
  // col 9: CumNQC (:400-410), sum over prefix sizes 2..n in order
  const double cum = ordered_sum((lane >= 1 && act) ? nqc_i : 0.0, k);
  const double cumnqc = k < 2 ? 0.0 : cum / (double)(k - 1);

  // per-element terms, one element per lane (transcendentals run once each)
  const double muhat = mu <= 0.0 ? 1.0 : mu;                  // SMV
  const double baseline = 1.0 / (0.01 > mu ? 0.01 : mu);      // WIG
  const double std_full = sqrt(var_full);                     // RSD
  const double x0 = readlane_f64(x, 0);
  const double thr = x0 * 0.5;                                // SigmaX
  double t_smv = 0.0, t_snqc = 0.0, t_skew = 0.0, t_wig = 0.0, t_uw = 0.0, t_w = 0.0;
  if (act) {
    if (x > 0.0) {
      t_smv = x * fabs(log(x / muhat));
      const double del = x - mu;
      const double prod = pow(1.0, 0.33) * pow((del * del) / x, 0.33);
      t_snqc = pow(prod, 0.33);
    }
    t_skew = pow((x - mu) / std_full, 3.0);
    t_wig = x - baseline;
    if (lane < 20) {  // UEF DCG weights (:349-363)
      t_w = 1.0 / (log((double)(lane + 2)) / log(2.0));
      t_uw = x * t_w;
    }
  }
  // Java adds the x <= 0 terms of SMV / SNQC as "skip": adding +0.0 is the same.
  const double smv = ordered_sum(t_smv, k);
  const double wig = ordered_sum(t_wig, k);
  const double skew = ordered_sum(t_skew, k);
  const double snqc = ordered_sum(t_snqc, k);
  const int ku = k < 20 ? k : 20;
  const double util = ordered_sum(t_uw, ku);
  const double wsum = ordered_sum(t_w, ku);
  // col 4: SigmaX (:299-319): compensated mean / variance of {x >= thr} in order
  const bool inF = act && x >= thr;
  const uint64_t fmask = ballot(inF);
  const int nf = __popcll(fmask);
  double sigmax = 0.0;
  if (k >= 2 && nf >= 2) {
    Kahan kf;
    kahan_init(kf);
    for (int j = 0; j < k; ++j)
      if ((fmask >> j) & 1ull) kahan_add(kf, readlane_f64(x, j));
    const double mf = kahan_final(kf) / (double)nf;
    const double dv = x - mf;
    const double t = dv * dv;
    Kahan kfv;
    kahan_init(kfv);
    for (int j = 0; j < k; ++j)
      if ((fmask >> j) & 1ull) kahan_add(kfv, readlane_f64(t, j));
    sigmax = sqrt(kahan_final(kfv) / (double)nf);
  }
  const double mx = wave_max(act ? x : -INFINITY);
  const double mn = wave_min(act ? x : INFINITY);
  double res[kQppCols];
  res[0] = nqc;
  res[1] = smv / (double)k;
  res[2] = wig / (double)(numTerms * k);
  res[3] = sigmamax;
  res[4] = sigmax;
  res[5] = (k < 3 || std_full < 1e-10) ? 0.0 : skew / (double)k;
  res[6] = util / wsum;
  res[7] = text_feat[2 * q];
  res[8] = text_feat[2 * q + 1];
  res[9] = cumnqc;
  res[10] = mu <= 0.0 ? 0.0 : snqc / (double)k;
  const double range = mx - mn;
  res[11] = (k < 2 || !(range > 0.0)) ? 0.0 : log(1.0 + 1.0 / range);
  res[12] = res[11];
  double v = 0.0;
#pragma unroll
  for (int c = 0; c < kQppCols; ++c)
    if (lane == c) v = res[c];
  if (lane < kQppCols) o[lane] = v;
}

// Column min / -max over present queries; one workgroup per (retriever, column).
__global__ __launch_bounds__(256) void qpp_colminmax_kernel(
    const double* __restrict__ raw, const int64_t* __restrict__ list_off, int64_t Q, int32_t R,
    double* __restrict__ mm) {
  __shared__ double smin[4], smax[4];
  const int rc = blockIdx.x;  // r * 13 + c
  const int r = rc / kQppCols, c = rc % kQppCols;
  double vmin = INFINITY, vmax = -INFINITY;
  for (int64_t q = threadIdx.x; q < Q; q += blockDim.x) {
    const int64_t l = q * R + r;
    if (list_off[l + 1] > list_off[l]) {
      const double v = raw[l * kQppCols + c];
      vmin = fmin(vmin, v);
      vmax = fmax(vmax, v);
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

// Normalise (src/qpp.py:356-372), round as "%.6f" (src/qpp.py:333), and derive
// the fusion weight the .qpp text round trip gives (src/fusion.py:150-158).
__global__ __launch_bounds__(256) void qpp_normalize_kernel(
    const double* __restrict__ raw, const double* __restrict__ mm,
    const int64_t* __restrict__ list_off, int64_t Q, int32_t R, int32_t mode, int32_t qpp_index,
    double* __restrict__ norm_out, int64_t* __restrict__ micro_out, double* __restrict__ w_out) {
  const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // list index q*R + r
  if (l >= Q * R) return;
  const int r = (int)(l % R);
  const bool present = list_off[l + 1] > list_off[l];
  double wsum = 0.0, wsel = 0.0;
  for (int c = 0; c < kQppCols; ++c) {
    const double x = raw[l * kQppCols + c];
    double v = x;
    if (mode == 1) {
      const double vmin = mm[r * kQppCols + c];
      const double vmax = -mm[R * kQppCols + r * kQppCols + c];
      const double scale = vmax > vmin ? vmax - vmin : 1.0;
      v = scale > 0.0 ? (x - vmin) / scale : 0.0;
    }
    if (!present) v = 0.0;
    const long long m = round6(v);
    if (norm_out) norm_out[l * kQppCols + c] = v;
    if (micro_out) micro_out[l * kQppCols + c] = m;
    const double back = (double)m / 1e6;  // float("%.6f") of the written text
    wsum += back;                          // Python sum(): left to right
    if (c == qpp_index) wsel = back;
  }
  if (w_out) w_out[l] = qpp_index < 0 ? wsum / (double)kQppCols : wsel;
}

hipError_t qpp_raw_launch(const double* score, const int64_t* list_off, int64_t Q, int32_t R,
                          int32_t top_k, const int32_t* nt, const double* tf, double* out,
                          hipStream_t st) {
  const int64_t L = Q * R;
  if (L == 0) return hipSuccess;
  const unsigned grid = (unsigned)((L + 3) / 4);
  hipLaunchKernelGGL(qpp_raw_kernel, dim3(grid), dim3(kQppBlock), 0, st, score, list_off, L, R,
                     top_k, nt, tf, out);
  return hipGetLastError();
}

hipError_t qpp_colminmax_launch(const double* raw, const int64_t* list_off, int64_t Q, int32_t R,
                                double* mm, hipStream_t st) {
  hipLaunchKernelGGL(qpp_colminmax_kernel, dim3(R * kQppCols), dim3(256), 0, st, raw, list_off, Q,
                     R, mm);
  return hipGetLastError();
}

hipError_t qpp_normalize_launch(const double* raw, const double* mm, const int64_t* list_off,
                                int64_t Q, int32_t R, int32_t mode, int32_t qpp_index,
                                double* norm_out, int64_t* micro_out, double* w_out,
                                hipStream_t st) {
  const int64_t L = Q * R;
  if (L == 0) return hipSuccess;
  hipLaunchKernelGGL(qpp_normalize_kernel, dim3((unsigned)((L + 255) / 256)), dim3(256), 0, st,
                     raw, mm, list_off, Q, R, mode, qpp_index, norm_out, micro_out, w_out);
  return hipGetLastError();
}

}  // namespace qf
