// qf_qpp.hip — score-distribution QPP predictors, one wavefront per list (gfx950).
//
// Replaces QPPBridge.computeQPPScores (src/qpp/java/qpp/QPPBridge.java:134-191)
// — formerly a JVM subprocess fed JSON (src/qpp.py:117-171) — and the driver's
// per-column min-max normalisation (src/qpp.py:340-374) + "%.6f" write-back
// (src/qpp.py:329-334) + get_qpp_weight (src/fusion.py:116-158).
//
// k = min(50, n) <= 64 values per list.  A workgroup takes 8 lists, one wave
// each: lane i holds rsv[i] for the per-element terms (every transcendental
// runs once per element) and owns prefix rsv[0..i] for the prefix statistics
// (SigmaMax, CumNQC).  Java's sequential summation order is reproduced
// exactly: every sum Java forms left to right is a serial chain here too, and
// every DoubleStream.average() is the JDK's compensated (Kahan) sum.  The
// chains of the 8 lists run batched (lane = list, or list x chain), so the
// serial work costs one lane each, not a whole wave; the chains that need only
// rsv (prefix sums, SigmaX) run on two waves at once, and everything that is not
// a chain (computeFinalSum's check, the divisions, UEF's weight sums) is taken
// off them.
#include "qf_common.h"
#include "qf_internal.h"
#include "qf_lists.h"

namespace qf {

// UEF's DCG weights 1 / (ln(i + 2) / ln 2), i < 20 (QPPBridge.java:349-363), computed
// with the host libm as the C restatement computes them (python -c: math.log).
__constant__ double kUefWeight[20] = {
    0x1.0000000000000p+0,
    0x1.430939835353dp-1,
    0x1.0000000000000p-1,
    0x1.b903469050f73p-2,
    0x1.8c23246dc0aa0p-2,
    0x1.6cc193acea9b5p-2,
    0x1.5555555555555p-2,
    0x1.430939835353dp-2,
    0x1.34413509f79fep-2,
    0x1.28009c1dd6453p-2,
    0x1.1da3383416063p-2,
    0x1.14b94f8d9641fp-2,
    0x1.0cf3ffed2d6acp-2,
    0x1.0619dc46d3e15p-2,
    0x1.0000000000000p-2,
    0x1.f50b57eac5883p-3,
    0x1.eb22cc68aa6e3p-3,
    0x1.e21e1180c5dabp-3,
    0x1.d9dcd21439834p-3,
    0x1.d244c78367a0dp-3};
// Their left-to-right sums from 0.0 (the loop's `weightSum += w`): kUefWeightSum[n-1]
// is the sum of the first n weights, so no chain of the kernel has to form it.
__constant__ double kUefWeightSum[20] = {
    0x1.0000000000000p+0,
    0x1.a1849cc1a9a9ep+0,
    0x1.10c24e60d4d4fp+1,
    0x1.47e2b732def3dp+1,
    0x1.79671bc097091p+1,
    0x1.a6ff4e36345c8p+1,
    0x1.d1a9f8e0df073p+1,
    0x1.fa0b20114971bp+1,
    0x1.1049a3594432dp+2,
    0x1.22c9ad1b21972p+2,
    0x1.34a3e09e62f78p+2,
    0x1.45ef75973c5bap+2,
    0x1.56beb5960f325p+2,
    0x1.6720535a7c706p+2,
    0x1.7720535a7c706p+2,
    0x1.86c8ae19d29cap+2,
    0x1.9621c47d17f01p+2,
    0x1.a532b5091e1eep+2,
    0x1.b4019b99bfeb0p+2,
    0x1.c293c1d5db280p+2};

// SNQC's pow(pow(1, 0.33) * pow(y, 0.33), 0.33) = y^(0.33 * 0.33) for y >= 0, as one
// exp(0.1089 ln y): within a few ulp of the nested pows (Java's Math.pow is itself a
// 1-ulp approximation; pow(1.0, 0.33) == 1.0 exactly), at a sixth of their instructions.
__device__ __forceinline__ double snqc_term(double y) { return exp((0.33 * 0.33) * log(y)); }

// x^3 with one rounding of the square carried (fma): ~1 ulp, like pow(x, 3.0).
__device__ __forceinline__ double cube(double x) {
  const double sq = x * x;
  const double lo = fma(x, x, -sq);
  return fma(sq, x, lo * x);
}

// A workgroup takes kQppLists lists, one wavefront each.  The per-element work is
// lane parallel inside the list's wave (lane i holds rsv[i]); the sums Java forms
// left to right are serial chains, and those run batched: one wave, one lane per
// (list, chain), so a chain costs one lane of one instruction instead of a whole
// wave's.
//
// SigmaMax and CumNQC (QPPBridge.java:269-293, 400-410) need the population
// variance of every prefix rsv[0..i].  Java recomputes each from scratch (a
// compensated prefix mean, then a compensated / simple sum of squared deviations
// around it): O(k^2).  Here one Welford chain per list carries the running mean
// and M2, so every prefix variance costs one step, O(k) — the values differ from
// Java's order by rounding only (<= 1.2e-13 relative over C2's and the section
// 8(d) generator's lists, tools/qpp_ok_study.py; no "%.6f" .qpp value changes).
// Every other column keeps Java's exact order: NQC (col 0) and RSD's variance
// (col 5, the default fusion weight) are the full-list sums of (x - mu)^2, simple
// and compensated, and RSD's skewness terms follow them.
//
// Phases (workgroup barriers between them):
//   B  chains over rsv: the compensated full-list sum (-> mu), SigmaX pass 1,
//      the Welford prefix variances (-> SigmaMax, CumNQC)   [waves 0, 1, 2]
//   C  per element: SMV / WIG / SNQC / UEF terms, (x - mu)^2 [every wave]
//   D  chains: the five simple sums, SigmaX pass 2, the compensated sum of
//      (x - mu)^2 (-> RSD's std)                           [waves 0, 1, 2]
//   E  per element: ((x - mu) / std)^3                      [every wave]
//   F  chain: the skewness sum                              [wave 0]

// A chain's next kBatch values read together: volatile, so the compiler cannot sink
// each read into its predicated step (it did: one exposed LDS latency per step of
// every serial chain — 50 per chain, the workgroup's critical path), and the reads'
// latency overlaps the previous batch's arithmetic.
constexpr int kBatch = 10;
__device__ __forceinline__ void lds_batch(const double* row, int j0, double (&b)[kBatch]) {
  typedef __attribute__((address_space(3))) const volatile double lds_f64;
  lds_f64* r = (lds_f64*)(__attribute__((address_space(3))) const double*)row;
#pragma unroll
  for (int t = 0; t < kBatch; ++t) b[t] = r[j0 + t];
}

constexpr int kQppLists = 8;
constexpr int kQppBlock = 64 * kQppLists;
constexpr int kRows = 5;     // smv, wig, snqc, uw, (x - mu)^2; then the skew terms
constexpr int kRow = 65;     // padded LDS row (doubles)
constexpr int kQppK = 50;    // k = min(50, n), QPPBridge.java:141

__global__ __launch_bounds__(kQppBlock, 8) void qpp_raw_kernel(
    const double* __restrict__ score, const int64_t* __restrict__ list_off, int64_t n_lists,
    int32_t R, int32_t top_k, const int32_t* __restrict__ num_terms,
    const double* __restrict__ text_feat, double* __restrict__ out) {
  __shared__ double s_x[kQppLists][kRow];          // rsv (float32-rounded)
  __shared__ double s_t[kQppLists][kRows][kRow];   // per-element terms of the chains
  __shared__ double s_res[kQppLists][kRows];       // simple chain sums (D)
  __shared__ double s_mu[kQppLists], s_cum[kQppLists], s_vmax[kQppLists];
  __shared__ double s_var[kQppLists], s_skew[kQppLists];
  __shared__ double s_sigmax[kQppLists];
  __shared__ double s_mf[kQppLists];  // SigmaX's compensated mean over F (pass 1)
  __shared__ unsigned long long s_fmask[kQppLists];
  __shared__ int s_k[kQppLists];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t l = block_id() * kQppLists + w;
  const bool lv = l < n_lists;  // every wave stays for the barriers
  int k = 0;
  int64_t a = 0;
  if (lv) {
    a = list_off[l];
    int64_t n64 = list_off[l + 1] - a;
    if (top_k > 0 && n64 > top_k) n64 = top_k;  // sorted(...)[:top_k], src/qpp.py:305
    k = n64 < 50 ? (int)n64 : 50;                // QPPBridge.java:141
  }
  const bool act = lane < k;
  // the query's inputs issued with the scores (one latency, not three)
  // (unconditional: q = 0 for a padding wave, whose values go unused)
  const int64_t q = lv ? l / R : 0;
  const int nt_raw = num_terms[q];
  const double tf0 = text_feat[2 * q], tf1 = text_feat[2 * q + 1];
  const double uefw = kUefWeight[lane < 20 ? lane : 0];          // UEF's DCG weight
  const double wsum = kUefWeightSum[(k < 20 ? (k > 0 ? k : 1) : 20) - 1];
  // float32 rounding of the JSON value (Gson getAsFloat), then widened.
  const double x = act ? (double)(float)score[a + lane] : 0.0;
  s_x[w][lane] = x;
  // col 4: SigmaX (:299-319) takes {x >= 0.5 x0} in order
  const double thr = __shfl(x, 0, 64) * 0.5;
  const uint64_t fmask = ballot(act && x >= thr);
  if (lane == 0) {
    s_k[w] = k;
    s_fmask[w] = fmask;
  }
  __syncthreads();
  QF_STOP(31, [&] { return (uint32_t)__double2loint(x) + nt_raw + __double2loint(tf0 + tf1); },
          if (_qf_acc == 12345u && lv) out[l * kQppCols] = 0.0; return;);

  // ---- B (lane = list): the chains that need only rsv, on three waves at once.
  // The serial loops run to kQppK unrolled (rows are kRow long; values past k
  // unused), only the arithmetic predicated; every sum keeps its order.  The
  // chains are the workgroup's critical path (its other waves wait at the barrier)
  // while the CU's other workgroups keep the SIMD busy: the chain waves run at
  // raised issue priority (s_setprio), so each dependent step issues as soon as its
  // operands are ready instead of queueing behind other waves' instructions.
  if (w <= 2) __builtin_amdgcn_s_setprio(3);
  if (w == 0 && lane < kQppLists) {
    // Arrays.stream(rsvs).average(): the JDK's compensated sum / n
    const int kl = s_k[lane];
    Kahan kp;
    kahan_init(kp);
#pragma unroll
    for (int j0 = 0; j0 < kQppK; j0 += kBatch) {
      double b[kBatch];
      lds_batch(s_x[lane], j0, b);
#pragma unroll
      for (int t = 0; t < kBatch; ++t)
        if (j0 + t < kl) kahan_add(kp, b[t]);
    }
    s_mu[lane] = kl > 0 ? div_int(kahan_final(kp), kl) : 0.0;
  } else if (w == 1 && lane < kQppLists) {
    // SigmaX, pass 1: the compensated mean over F.  Pass 2 (the compensated mean of
    // (x - mean)^2) runs in D beside the left-to-right sums.
    const int kl = s_k[lane];
    const uint64_t fm = s_fmask[lane];
    const int nf = __popcll(fm);
    double mf = 0.0;
    if (kl >= 2 && nf >= 2) {
      Kahan kf;
      kahan_init(kf);
#pragma unroll
      for (int j0 = 0; j0 < kQppK; j0 += kBatch) {
        double b[kBatch];
        lds_batch(s_x[lane], j0, b);
#pragma unroll
        for (int t = 0; t < kBatch; ++t)
          if (j0 + t < kl && ((fm >> (j0 + t)) & 1ull)) kahan_add(kf, b[t]);
      }
      mf = div_int(kahan_final(kf), nf);
    }
    s_mf[lane] = mf;
  } else if (w == 2 && lane < kQppLists) {
    // Welford: mean_i = mean_{i-1} + d / (i + 1), M2_i = M2_{i-1} + d (x_i - mean_i),
    // var_i = M2_i / (i + 1); SigmaMax takes the largest var_i of the prefixes of 2..k
    // elements (sqrt is monotone: the max of the sigmas is the sigma of the max),
    // CumNQC their sum in prefix order (the NQC of a prefix is its variance).
    const int kl = s_k[lane];
    double mean = 0.0, m2 = 0.0, cum = 0.0, vmax = 0.0;
#pragma unroll
    for (int j0 = 0; j0 < kQppK; j0 += kBatch) {
      double b[kBatch];
      lds_batch(s_x[lane], j0, b);
#pragma unroll
      for (int t = 0; t < kBatch; ++t) {
        const int j = j0 + t;
        const double inv = 1.0 / (double)(j + 1);  // a literal: the loop is unrolled
        if (j < kl) {
          const double d = b[t] - mean;
          mean = fma(d, inv, mean);
          m2 = fma(d, b[t] - mean, m2);
          if (j >= 1) {
            const double var = m2 * inv;
            cum += var;
            vmax = fmax(vmax, var);
          }
        }
      }
    }
    s_cum[lane] = cum;
    s_vmax[lane] = vmax;
  }
  if (w <= 2) __builtin_amdgcn_s_setprio(0);
  __syncthreads();
  QF_STOP(32, [&] { return (uint32_t)__double2loint(s_mu[w] + s_cum[w] + s_vmax[w] + s_mf[w]) + nt_raw + __double2loint(tf0 + tf1); },
          if (_qf_acc == 12345u && lv) out[l * kQppCols] = 0.0; return;);

  // ---- C (each list's wave): the per-element terms (transcendentals once each)
  const int numTerms = nt_raw > 1 ? nt_raw : 1;  // Math.max(1, terms.length)
  const double mu = s_mu[w];
  const double muhat = mu <= 0.0 ? 1.0 : mu;                  // SMV
  const double baseline = 1.0 / (0.01 > mu ? 0.01 : mu);      // WIG
  double t_smv = 0.0, t_snqc = 0.0, t_wig = 0.0, t_uw = 0.0, t_d2 = 0.0;
  if (act) {
    const double del = x - mu;
    t_d2 = del * del;  // Math.pow(s - mean, 2) == s*s exactly
    if (x > 0.0) {
      t_smv = x * fabs(log(x / muhat));
      t_snqc = snqc_term(t_d2 / x);
    }
    t_wig = x - baseline;
    if (lane < 20) t_uw = x * uefw;  // UEF (:349-363)
  }
  // Java adds the x <= 0 terms of SMV / SNQC as "skip": adding +0.0 is the same.
  s_t[w][0][lane] = t_smv;
  s_t[w][1][lane] = t_wig;
  s_t[w][2][lane] = t_snqc;
  s_t[w][3][lane] = t_uw;
  s_t[w][4][lane] = t_d2;
  const double mx = wave_max(act ? x : -INFINITY);
  const double mn = wave_min(act ? x : INFINITY);
  __syncthreads();
  QF_STOP(33, [&] { return (uint32_t)__double2loint(mx + mn) + nt_raw + __double2loint(tf0 + tf1 + uefw + wsum); },
          if (_qf_acc == 12345u && lv) out[l * kQppCols] = 0.0; return;);

  // ---- D: the left-to-right sums (wave 0, lane = list * 8 + row: SMV, WIG, SNQC,
  // UEF, NQC's simple sum of (x - mu)^2), SigmaX pass 2 (wave 1) and RSD's
  // compensated mean of (x - mu)^2 (wave 2), all lists at once
  if (w <= 2) __builtin_amdgcn_s_setprio(3);
  if (w == 0 && (lane & 7) < kRows) {
    const int ll = lane >> 3, c = lane & 7;
    const int kl = s_k[ll];
    const int len = c == 3 ? (kl < 20 ? kl : 20) : kl;
    const double* row = s_t[ll][c];
    double acc = 0.0;
#pragma unroll
    for (int j0 = 0; j0 < kQppK; j0 += kBatch) {
      double b[kBatch];
      lds_batch(row, j0, b);
#pragma unroll
      for (int t = 0; t < kBatch; ++t)
        if (j0 + t < len) acc += b[t];
    }
    s_res[ll][c] = acc;
  } else if (w == 1 && lane < kQppLists) {  // SigmaX, pass 2 (pass 1 in B)
    const int kl = s_k[lane];
    const uint64_t fm = s_fmask[lane];
    const int nf = __popcll(fm);
    double sigmax = 0.0;
    if (kl >= 2 && nf >= 2) {
      const double mf = s_mf[lane];
      Kahan kfv;
      kahan_init(kfv);
#pragma unroll
      for (int j0 = 0; j0 < kQppK; j0 += kBatch) {
        double b[kBatch];
        lds_batch(s_x[lane], j0, b);
#pragma unroll
        for (int t = 0; t < kBatch; ++t) {
          const double dv = b[t] - mf;
          if (j0 + t < kl && ((fm >> (j0 + t)) & 1ull)) kahan_add(kfv, dv * dv);
        }
      }
      sigmax = sqrt(div_int(kahan_final(kfv), nf));
    }
    s_sigmax[lane] = sigmax;
  } else if (w == 2 && lane < kQppLists) {  // RSD (:320-344): std of the full list
    const int kl = s_k[lane];
    Kahan kv;
    kahan_init(kv);
#pragma unroll
    for (int j0 = 0; j0 < kQppK; j0 += kBatch) {
      double b[kBatch];
      lds_batch(s_t[lane][4], j0, b);
#pragma unroll
      for (int t = 0; t < kBatch; ++t)
        if (j0 + t < kl) kahan_add(kv, b[t]);
    }
    s_var[lane] = kl > 0 ? div_int(kahan_final(kv), kl) : 0.0;
  }
  if (w <= 2) __builtin_amdgcn_s_setprio(0);
  __syncthreads();
  QF_STOP(34, [&] { return (uint32_t)__double2loint(mx + mn + s_res[w][0] + s_var[w] + s_sigmax[w]) + nt_raw + __double2loint(tf0 + tf1 + uefw + wsum); },
          if (_qf_acc == 12345u && lv) out[l * kQppCols] = 0.0; return;);

  // ---- E (each list's wave): RSD's skewness terms, over the row D has consumed
  const double std_full = sqrt(s_var[w]);
  s_t[w][4][lane] = act ? cube((x - mu) / std_full) : 0.0;
  __syncthreads();
  QF_STOP(35, [&] { return (uint32_t)__double2loint(mx + mn + s_res[w][0] + s_var[w] + s_sigmax[w]) + nt_raw + __double2loint(tf0 + tf1 + uefw + wsum); },
          if (_qf_acc == 12345u && lv) out[l * kQppCols] = 0.0; return;);

  // ---- F (wave 0, lane = list): the skewness sum
  if (w == 0 && lane < kQppLists) {
    __builtin_amdgcn_s_setprio(3);
    const int kl = s_k[lane];
    double acc = 0.0;
#pragma unroll
    for (int j0 = 0; j0 < kQppK; j0 += kBatch) {
      double b[kBatch];
      lds_batch(s_t[lane][4], j0, b);
#pragma unroll
      for (int t = 0; t < kBatch; ++t)
        if (j0 + t < kl) acc += b[t];
    }
    s_skew[lane] = acc;
    __builtin_amdgcn_s_setprio(0);
  }
  __syncthreads();

  if (!lv) return;
  double* o = out + l * kQppCols;
  if (k == 0) {  // empty map -> every column 0.0 (src/qpp.py:321)
    if (lane < kQppCols) o[lane] = 0.0;
    return;
  }
  const double smv = s_res[w][0], wig = s_res[w][1], snqc = s_res[w][2], util = s_res[w][3];
  const double sq = s_res[w][4], skew = s_skew[w];
  double res[kQppCols];
  res[0] = div_int(sq, k);                                             // NQC (:202-216)
  res[1] = div_int(smv, k);
  res[2] = div_int(wig, numTerms * k);
  res[3] = k < 2 ? 0.0 : sqrt(s_vmax[w]) / sqrt((double)numTerms);    // SigmaMax
  res[4] = s_sigmax[w];
  res[5] = (k < 3 || std_full < 1e-10) ? 0.0 : div_int(skew, k);
  res[6] = util / wsum;
  res[7] = tf0;
  res[8] = tf1;
  res[9] = k < 2 ? 0.0 : div_int(s_cum[w], k - 1);                    // CumNQC
  res[10] = mu <= 0.0 ? 0.0 : div_int(snqc, k);
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
  qpp_colminmax_block(raw, list_off, Q, R, mm, (int)blockIdx.x);
}

// ---- zscore statistics: numpy's mean / std of each column --------------------
//
// src/qpp.py:358-359 takes arr.mean() and arr.std() of a float64 column.  numpy
// sums a contiguous float64 array as acc = 0.0; acc += pairwise(chunk) over
// 8192-element chunks (the ufunc buffer), pairwise() being its fixed recursion
// (n < 8: left to right from -0.0; n <= 128: 8 interleaved accumulators; else
// split at n/2 rounded down to a multiple of 8).  std = sqrt(sum((x - mean)^2) / n)
// with mean = sum(x) / n.  Both are reproduced exactly: one workgroup per
// (retriever, column) gathers the present rows of a chunk into LDS, sums the
// recursion's leaves in parallel and combines them in the recursion's order.
constexpr int kNpChunk = 8192;
constexpr int kNpLeaves = 128;  // leaves hold 64..128 elements of a full chunk

struct NpFrame {
  int lo, n, st;
  double left;
};

// Walks pairwise(0, m) depth first.  LEAF(lo, n) returns the sum of a leaf.
template <class LEAF>
__device__ double np_pairwise_walk(int m, LEAF leaf) {
  NpFrame f[12];
  int sp = 0;
  f[0] = {0, m, 0, 0.0};
  double ret = 0.0;
  while (true) {
    if (f[sp].n <= 128) {
      ret = leaf(f[sp].lo, f[sp].n);
      while (true) {  // deliver ret upwards
        if (sp == 0) return ret;
        --sp;
        if (f[sp].st == 1) {
          f[sp].left = ret;
          f[sp].st = 2;
          int n2 = f[sp].n / 2;
          n2 -= n2 % 8;
          f[sp + 1] = {f[sp].lo + n2, f[sp].n - n2, 0, 0.0};
          ++sp;
          break;
        }
        ret = f[sp].left + ret;
      }
    } else {
      f[sp].st = 1;
      int n2 = f[sp].n / 2;
      n2 -= n2 % 8;
      f[sp + 1] = {f[sp].lo, n2, 0, 0.0};
      ++sp;
    }
  }
}

// numpy's leaf: DOUBLE_pairwise_sum for n <= 128.
__device__ double np_leaf_sum(const double* a, int n) {
  if (n < 8) {
    double res = -0.0;
    for (int i = 0; i < n; ++i) res += a[i];
    return res;
  }
  double r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}

__global__ __launch_bounds__(256) void qpp_colmeanstd_kernel(
    const double* __restrict__ raw, const int64_t* __restrict__ list_off, int64_t Q, int32_t R,
    double* __restrict__ st) {
  __shared__ double s_val[kNpChunk];
  __shared__ double s_leaf[kNpLeaves];
  __shared__ int s_llo[kNpLeaves], s_ln[kNpLeaves];
  __shared__ int s_nleaf, s_fill, s_take;
  __shared__ int s_wcnt[4];
  __shared__ double s_acc;
  const int rc = blockIdx.x;  // r * 13 + c
  const int r = rc / kQppCols, c = rc % kQppCols;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  double mean = 0.0;
  int64_t n_total = 0;
  for (int pass = 0; pass < 2; ++pass) {
    if (tid == 0) s_acc = 0.0;
    int64_t cursor = 0;  // next row to scan
    n_total = 0;
    while (true) {
      // ---- gather the next <= kNpChunk present rows (in row order) into s_val
      if (tid == 0) s_fill = 0;
      __syncthreads();
      while (cursor < Q && s_fill < kNpChunk) {
        const int64_t row = cursor + tid;
        bool pres = false;
        if (row < Q) {
          const int64_t l = row * R + r;
          pres = list_off[l + 1] > list_off[l];
        }
        const uint64_t b = ballot(pres);
        if (lane == 0) s_wcnt[wid] = __popcll(b);
        __syncthreads();
        int before = (int)mbcnt(b);
        for (int w = 0; w < wid; ++w) before += s_wcnt[w];
        const int total = s_wcnt[0] + s_wcnt[1] + s_wcnt[2] + s_wcnt[3];
        const int fill = s_fill, room = kNpChunk - fill;
        if (pres && before < room) {
          double v = raw[(row * R + r) * kQppCols + c];
          if (pass == 1) {
            const double d = v - mean;  // numpy: x = arr - arrmean; x * x
            v = d * d;
          }
          s_val[fill + before] = v;
          if (before == room - 1) s_take = tid + 1;  // the row that fills the chunk
        }
        __syncthreads();
        if (total <= room) {
          cursor += 256;
          if (tid == 0) s_fill = fill + total;
        } else {
          cursor += s_take;
          if (tid == 0) s_fill = kNpChunk;
        }
        __syncthreads();
      }
      const int m = s_fill;
      if (m == 0) break;
      n_total += m;
      // ---- leaves of pairwise(0, m) in recursion order, summed in parallel
      if (tid == 0) {
        int k = 0;
        np_pairwise_walk(m, [&](int lo, int n) {
          s_llo[k] = lo;
          s_ln[k] = n;
          ++k;
          return 0.0;
        });
        s_nleaf = k;
      }
      __syncthreads();
      if (tid < s_nleaf) s_leaf[tid] = np_leaf_sum(s_val + s_llo[tid], s_ln[tid]);
      __syncthreads();
      if (tid == 0) {
        int k = 0;
        const double chunk = np_pairwise_walk(m, [&](int, int) { return s_leaf[k++]; });
        s_acc = s_acc + chunk;
      }
      __syncthreads();
      if (m < kNpChunk) break;
    }
    const double sum = s_acc;
    if (pass == 0) mean = sum / (double)n_total;
    else if (tid == 0) {
      const double sd = sqrt(sum / (double)n_total);
      st[rc] = n_total ? mean : 0.0;
      st[R * kQppCols + rc] = sd > 0.0 ? sd : 1.0;  // arr.std() if arr.std() > 0 else 1.0
    }
    __syncthreads();
  }
}

// Normalise (src/qpp.py:356-372), round as "%.6f" (src/qpp.py:333), and derive
// the fusion weight the .qpp text round trip gives (src/fusion.py:150-158).
__global__ __launch_bounds__(256) void qpp_normalize_kernel(
    const double* __restrict__ raw, const double* __restrict__ mm,
    const int64_t* __restrict__ list_off, int64_t Q, int32_t R, int32_t mode, int32_t qpp_index,
    double* __restrict__ norm_out, int64_t* __restrict__ micro_out, double* __restrict__ w_out) {
  const int64_t l = block_id() * blockDim.x + threadIdx.x;  // list index q*R + r
  if (l >= Q * R) return;
  const int r = (int)(l % R);
  const bool present = list_off[l + 1] > list_off[l];
  // every load in flight before the first use (one memory latency per thread)
  double xs[kQppCols], m0[kQppCols], m1[kQppCols];
#pragma unroll
  for (int c = 0; c < kQppCols; ++c) {
    xs[c] = raw[l * kQppCols + c];
    m0[c] = mode != 0 ? mm[r * kQppCols + c] : 0.0;
    m1[c] = mode != 0 ? mm[R * kQppCols + r * kQppCols + c] : 0.0;
  }
  double wsum = 0.0, wsel = 0.0;
#pragma unroll
  for (int c = 0; c < kQppCols; ++c) {
    const double v = qpp_norm_value(xs[c], m0[c], m1[c], mode, present);
    const long long m = round6(v);
    if (norm_out) norm_out[l * kQppCols + c] = v;
    if (micro_out) micro_out[l * kQppCols + c] = m;
    const double back = micro_back(m);     // the .qpp text read back
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
  hipLaunchKernelGGL(qpp_raw_kernel, grid_for((L + kQppLists - 1) / kQppLists), dim3(kQppBlock), 0,
                     st, score, list_off, L, R,
                     top_k, nt, tf, out);
  return hipGetLastError();
}

hipError_t qpp_colminmax_launch(const double* raw, const int64_t* list_off, int64_t Q, int32_t R,
                                double* mm, hipStream_t st) {
  hipLaunchKernelGGL(qpp_colminmax_kernel, dim3(R * kQppCols), dim3(256), 0, st, raw, list_off, Q,
                     R, mm);
  return hipGetLastError();
}

hipError_t qpp_colmeanstd_launch(const double* raw, const int64_t* list_off, int64_t Q,
                                 int32_t R, double* st, hipStream_t stm) {
  hipLaunchKernelGGL(qpp_colmeanstd_kernel, dim3(R * kQppCols), dim3(256), 0, stm, raw, list_off,
                     Q, R, st);
  return hipGetLastError();
}

hipError_t qpp_normalize_launch(const double* raw, const double* mm, const int64_t* list_off,
                                int64_t Q, int32_t R, int32_t mode, int32_t qpp_index,
                                double* norm_out, int64_t* micro_out, double* w_out,
                                hipStream_t st) {
  const int64_t L = Q * R;
  if (L == 0) return hipSuccess;
  hipLaunchKernelGGL(qpp_normalize_kernel, grid_for((L + 255) / 256), dim3(256), 0, st,
                     raw, mm, list_off, Q, R, mode, qpp_index, norm_out, micro_out, w_out);
  return hipGetLastError();
}

// Learned fusion's feature matrix from the normalised predictors' "%.6f" values:
// X[q, j*13 + c] = micro[(q*R + run_of_block[j])*13 + c] / 1e6 — the .qpp text
// read back (src/data_utils.py:262-293) and laid out per model retriever
// (src/fusion.py:421-427); a block whose run is -1 (a retriever the batch lacks)
// stays 0.0.  One thread per feature, coalesced writes.
__global__ __launch_bounds__(256) void qpp_features_kernel(const int64_t* __restrict__ micro,
                                                           int64_t Q, int32_t R, QppBlocks blk,
                                                           double* __restrict__ X) {
  const int64_t i = block_id() * blockDim.x + threadIdx.x;
  const int64_t F = (int64_t)blk.n * kQppCols;
  if (i >= Q * F) return;
  const int64_t q = i / F;
  const int f = (int)(i - q * F);
  const int j = f / kQppCols, c = f - j * kQppCols;
  const int r = blk.run[j];
  double v = 0.0;
  if (r >= 0) {
    const int64_t m = micro[(q * R + r) * kQppCols + c];
    v = (m > -0x7FFFFFFFll && m < 0x7FFFFFFFll) ? micro_to_f64((int32_t)m) : (double)m / 1e6;
  }
  X[i] = v;
}

hipError_t qpp_features_launch(const int64_t* micro, int64_t Q, int32_t R, const QppBlocks& blk,
                               double* X, hipStream_t st) {
  const int64_t n = Q * blk.n * kQppCols;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(qpp_features_kernel, grid_for((n + 255) / 256), dim3(256), 0, st, micro, Q,
                     R, blk, X);
  return hipGetLastError();
}

}  // namespace qf

