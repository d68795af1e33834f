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

__global__ __launch_bounds__(kQppBlock) void qpp_raw_kernel(
    const double* __restrict__ score, const int64_t* __restrict__ list_off, int64_t n_lists,
    int32_t R, int32_t top_k, const int32_t* __restrict__ num_terms,
    const double* __restrict__ text_feat, double* __restrict__ out) {
  __shared__ double xs_all[kQppBlock];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t l = (int64_t)blockIdx.x * (kQppBlock / 64) + wid;
  if (l >= n_lists) return;  // wave-uniform; no block barrier below
  double* xs = xs_all + wid * 64;
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
  // float32 rounding of the JSON value (Gson getAsFloat), then widened.
  const double x = lane < k ? (double)(float)score[a + lane] : 0.0;
  xs[lane] = x;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  const int nt_raw = num_terms[q];
  const int numTerms = nt_raw > 1 ? nt_raw : 1;  // Math.max(1, terms.length)

  // prefix Kahan means: lane i -> mean of rsv[0..i]
  Kahan kp;
  kahan_init(kp);
  for (int j = 0; j < k; ++j) {
    const double xj = xs[j];
    if (j <= lane) kahan_add(kp, xj);
  }
  const double mean_i = kahan_final(kp) / (double)(lane + 1);
  const double mu = __shfl(mean_i, k - 1, 64);  // Arrays.stream(rsvs).average()

  // prefix sums of squared deviations around each prefix mean:
  //   simple sum -> NQC of prefix (CumNQC, NQC), Kahan average -> SigmaMax
  Kahan kv;
  kahan_init(kv);
  double sq = 0.0;
  for (int j = 0; j < k; ++j) {
    const double xj = xs[j];
    if (j <= lane) {
      const double del = xj - mean_i;
      const double d2 = del * del;  // Math.pow(s - mean, 2) == s*s exactly
      sq += d2;
      kahan_add(kv, d2);
    }
  }
  const double nqc_i = sq / (double)(lane + 1);                    // computeNQC(prefix)
  const double sigma_i = sqrt(kahan_final(kv) / (double)(lane + 1));  // SigmaMax window std
  const double var_full = __shfl(kahan_final(kv) / (double)(lane + 1), k - 1, 64);

  // ---- col 0: NQC (QPPBridge.java:202-216)
  const double nqc = __shfl(nqc_i, k - 1, 64);
  // ---- col 3: SigmaMax (QPPBridge.java:269-293)
  double sm = (lane >= 1 && lane < k) ? sigma_i : 0.0;
  sm = wave_max(sm);
  const double sigmamax = k < 2 ? 0.0 : sm / sqrt((double)numTerms);
  // ---- col 9: CumNQC (QPPBridge.java:400-410): sequential over k = 2..n
  double cum = 0.0;
  for (int j = 1; j < k; ++j) cum += __shfl(nqc_i, j, 64);
  const double cumnqc = k < 2 ? 0.0 : cum / (double)(k - 1);

  // ---- sequential single-accumulator loops (uniform across lanes)
  const double muhat = mu <= 0.0 ? 1.0 : mu;                         // SMV
  const double baseline = 1.0 / (0.01 > mu ? 0.01 : mu);             // WIG
  const double std_full = sqrt(var_full);                            // RSD
  const double thr = xs[0] * 0.5;                                    // SigmaX
  double smv = 0.0, wig = 0.0, skew = 0.0, snqc = 0.0, mx = xs[0], mn = xs[0];
  Kahan kf;
  kahan_init(kf);
  int nf = 0;
  for (int j = 0; j < k; ++j) {
    const double xj = xs[j];
    if (xj > 0.0) smv += xj * fabs(log(xj / muhat));
    wig += (xj - baseline);
    skew += pow((xj - mu) / std_full, 3.0);
    if (xj > 0.0) {
      const double del = xj - mu;
      const double f2 = (del * del) / xj;
      const double prod = pow(1.0, 0.33) * pow(f2, 0.33);
      snqc += pow(prod, 0.33);
    }
    if (xj >= thr) { kahan_add(kf, xj); ++nf; }
    mx = fmax(mx, xj);
    mn = fmin(mn, xj);
  }
  // ---- col 4: SigmaX (QPPBridge.java:299-319)
  double sigmax = 0.0;
  if (k >= 2 && nf >= 2) {
    const double mf = kahan_final(kf) / (double)nf;
    Kahan kfv;
    kahan_init(kfv);
    for (int j = 0; j < k; ++j) {
      const double xj = xs[j];
      if (xj >= thr) {
        const double del = xj - mf;
        kahan_add(kfv, del * del);
      }
    }
    sigmax = sqrt(kahan_final(kfv) / (double)nf);
  }
  // ---- col 6: UEF (QPPBridge.java:349-363)
  double util = 0.0, wsum = 0.0;
  const int ku = k < 20 ? k : 20;
  const double ln2 = log(2.0);
  for (int i = 0; i < ku; ++i) {
    const double wgt = 1.0 / (log((double)(i + 2)) / ln2);
    util += xs[i] * wgt;
    wsum += wgt;
  }
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
