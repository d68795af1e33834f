/*
 * qpp_oracle.c — TEST INFRASTRUCTURE ONLY (CPU oracle; never linked into,
 * called by, or shipped with the product).
 *
 * Literal C restatement of QPPBridge.computeQPPScores and its 13 predictor
 * functions (src/qpp/java/qpp/QPPBridge.java:134-453), written as the Java
 * runs: each method recomputes its own statistics with its own loops, exactly
 * as the Java source does (no sharing of intermediate results, unlike the GPU
 * kernel), plus the driver's per-column min-max (src/qpp.py:340-374).
 *
 * Java details reproduced:
 *  - scores arrive as float (Gson getAsFloat, :67-70) and are widened to double;
 *    rsvs = first k = min(50, n) (:141-142);
 *  - DoubleStream.average() is the JDK's compensated sum
 *    (Collectors.sumWithCompensation / computeFinalSum, JDK 11-17 form);
 *  - Math.pow(x, 2) == x*x exactly (fdlibm special case), other pow via libm;
 *  - int arithmetic where Java uses int (numTerms * rsvs.length).
 * The text features (MaxIDF / avgidf proxies, numTerms) are host string work
 * and are passed in (oracle/text_oracle.py restates them).
 * The Java toolchain is absent in this image (no java/javac), so this
 * restatement is "parity unpinned" for the score-based columns; see DESIGN.md.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* Gson's getAsFloat of the number json.dumps wrote (QPPBridge.java:67-70,
 * src/qpp.py:130-147): Float.parseFloat(repr(d)) — repr is the shortest decimal
 * that reads back as d (the correctly rounded %.{p}g for the smallest such p),
 * and strtof rounds a decimal correctly.  (float)d differs only when d is
 * exactly halfway between two floats, so the text path runs only there and
 * outside the float normal range. */
static double java_float(double d) {
  uint64_t b;
  memcpy(&b, &d, 8);
  const unsigned e = (unsigned)((b >> 52) & 0x7FF);
  const int normal32 = e >= 1023 - 126 && e <= 1023 + 127;
  const int midpoint = (b & 0x1FFFFFFFull) == 0x10000000ull;
  if (!(midpoint || !normal32) || !isfinite(d) || d == 0.0) return (double)(float)d;
  char buf[64];
  for (int p = 1; p <= 17; ++p) {
    snprintf(buf, sizeof buf, "%.*g", p, d);
    if (strtod(buf, NULL) == d) break;
  }
  return (double)strtof(buf, NULL);
}

typedef struct { double s, c, simple; } kahan_t;

static void k_init(kahan_t* k) { k->s = 0.0; k->c = 0.0; k->simple = 0.0; }
static void k_add(kahan_t* k, double v) {
  double tmp = v - k->c;
  double sum = k->s;
  double velvel = sum + tmp;
  k->c = (velvel - sum) - tmp;
  k->s = velvel;
  k->simple += v;
}
static double k_final(const kahan_t* k) {
  double tmp = k->s + k->c;
  if (isnan(tmp) && isinf(k->simple)) return k->simple;
  return tmp;
}
/* Arrays.stream(a, 0, n).average().orElse(dflt) */
static double j_average(const double* a, int n, double dflt) {
  if (n <= 0) return dflt;
  kahan_t k; k_init(&k);
  for (int i = 0; i < n; ++i) k_add(&k, a[i]);
  return k_final(&k) / (double)n;
}

static double computeNQC(const double* r, int n) {
  if (n == 0) return 0.0;
  double mean = j_average(r, n, 0.0);
  double nqc = 0.0;
  for (int i = 0; i < n; ++i) { double del = r[i] - mean; nqc += del * del; }
  nqc /= n;
  return nqc * 1.0;
}
static double computeSMV(const double* r, int n) {
  if (n == 0) return 0.0;
  double muHat = j_average(r, n, 1.0);
  if (muHat <= 0) muHat = 1.0;
  double smv = 0.0;
  for (int i = 0; i < n; ++i)
    if (r[i] > 0) smv += r[i] * fabs(log(r[i] / muHat));
  return smv / n;
}
static double computeWIG(int numTerms, const double* r, int n) {
  if (n == 0) return 0.0;
  double avg = j_average(r, n, 1.0);
  double baseline = 1.0 / fmax(0.01, avg);
  double wig = 0.0;
  for (int i = 0; i < n; ++i) wig += (r[i] - baseline);
  return wig / (double)(numTerms * n);
}
static double computeSigmaMax(int numTerms, const double* r, int n) {
  if (n < 2) return 0.0;
  double maxStd = 0.0;
  double* tmp = malloc(sizeof(double) * (size_t)n);
  for (int i = 0; i < n; ++i) {
    int m = i + 1;
    if (m >= 2) {
      double mean = j_average(r, m, 0.0);
      for (int j = 0; j < m; ++j) { double d = r[j] - mean; tmp[j] = d * d; }
      double variance = j_average(tmp, m, 0.0);
      double sigma = sqrt(variance);
      maxStd = fmax(maxStd, sigma);
    }
  }
  free(tmp);
  return maxStd / sqrt((double)(numTerms > 1 ? numTerms : 1));
}
static double computeSigmaX(const double* r, int n) {
  if (n < 2) return 0.0;
  double threshold = r[0] * 0.5;
  double* f = malloc(sizeof(double) * (size_t)n);
  int nf = 0;
  for (int i = 0; i < n; ++i) if (r[i] >= threshold) f[nf++] = r[i];
  if (nf < 2) { free(f); return 0.0; }
  double mean = j_average(f, nf, 0.0);
  for (int i = 0; i < nf; ++i) { double d = f[i] - mean; f[i] = d * d; }
  double variance = j_average(f, nf, 0.0);
  free(f);
  return sqrt(variance);
}
static double computeRSD(const double* r, int n) {
  if (n < 3) return 0.0;
  double mean = j_average(r, n, 0.0);
  double* t = malloc(sizeof(double) * (size_t)n);
  for (int i = 0; i < n; ++i) { double d = r[i] - mean; t[i] = d * d; }
  double std = sqrt(j_average(t, n, 0.0));
  free(t);
  if (std < 1e-10) return 0.0;
  double skew = 0.0;
  for (int i = 0; i < n; ++i) skew += pow((r[i] - mean) / std, 3.0);
  return skew / n;
}
static double computeUEF(const double* r, int n) {
  if (n == 0) return 0.0;
  double utility = 0.0, weightSum = 0.0;
  int k = n < 20 ? n : 20;
  for (int i = 0; i < k; ++i) {
    double weight = 1.0 / (log((double)(i + 2)) / log(2.0));
    utility += r[i] * weight;
    weightSum += weight;
  }
  return utility / weightSum;
}
static double computeCumNQC(const double* r, int n) {
  if (n < 2) return 0.0;
  double cum = 0.0;
  for (int k = 2; k <= n; ++k) cum += computeNQC(r, k);
  return cum / (n - 1);
}
static double computeSNQC(const double* r, int n) {
  if (n == 0) return 0.0;
  double mean = j_average(r, n, 0.0);
  if (mean <= 0) return 0.0;
  double snqc = 0.0;
  for (int i = 0; i < n; ++i) {
    if (r[i] <= 0) continue;
    double d = r[i] - mean;
    double factor2 = (d * d) / r[i];
    double prod = pow(1.0, 0.33) * pow(factor2, 0.33);
    prod = pow(prod, 0.33);
    snqc += prod;
  }
  snqc /= n;
  return snqc * 1.0;
}
static double computeScoreSpread(const double* r, int n) {
  if (n < 2) return 0.0;
  double mx = r[0], mn = r[0];
  for (int i = 1; i < n; ++i) { mx = fmax(mx, r[i]); mn = fmin(mn, r[i]); }
  double range = mx - mn;
  return range > 0 ? log(1 + 1.0 / range) : 0.0;
}

/*
 * One row of 13 raw predictors per list.  score: doubles (as the driver holds
 * them, already sorted desc and truncated by the caller); the float32 rounding
 * happens here.  num_terms_raw / maxidf / avgidf per list.
 */
void oracle_qpp_raw(const double* score, const int64_t* list_off, int64_t n_lists,
                    const int32_t* num_terms_raw, const double* maxidf, const double* avgidf,
                    double* out) {
  double r[50];
  for (int64_t l = 0; l < n_lists; ++l) {
    int64_t n64 = list_off[l + 1] - list_off[l];
    double* o = out + l * 13;
    if (n64 <= 0) { for (int c = 0; c < 13; ++c) o[c] = 0.0; continue; }
    int k = n64 < 50 ? (int)n64 : 50;
    for (int i = 0; i < k; ++i) r[i] = java_float(score[list_off[l] + i]);
    int nt = num_terms_raw[l] > 1 ? num_terms_raw[l] : 1;
    o[0] = computeNQC(r, k);
    o[1] = computeSMV(r, k);
    o[2] = computeWIG(nt, r, k);
    o[3] = computeSigmaMax(nt, r, k);
    o[4] = computeSigmaX(r, k);
    o[5] = computeRSD(r, k);
    o[6] = computeUEF(r, k);
    o[7] = maxidf[l];
    o[8] = avgidf[l];
    o[9] = computeCumNQC(r, k);
    o[10] = computeSNQC(r, k);
    o[11] = computeScoreSpread(r, k);
    o[12] = computeScoreSpread(r, k);
  }
}
