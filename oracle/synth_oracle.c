/* synth_oracle.c — TEST INFRASTRUCTURE ONLY: a CPU regeneration of qf_synth_runs_nq
 * (csrc/qf_synth.hip, SURVEY.md §8(d)'s synthetic runs), operation for operation, so
 * a GPU test can check the device generator bit for bit on a sample of queries.
 * Compiled with -ffp-contract=off (oracle/Makefile), like the library.
 *
 * Per list (q, r): K positions; position i draws pool membership and its score from
 * Philox4x32-10 (key (seed, stream), counter (i, r, q_lo, q_hi)); pool positions take
 * pool ids a + pi(k), the others g(k) skipping the pool block; the K scores are
 * sorted descending and get 1e-6 * (K - 1 - rank); the query's judged documents are
 * planted with probability p_r at Geometric(0.15) ranks.  See qf_synth.hip.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define NQ_CORPUS 2681468u

typedef struct { uint32_t x[4]; } ph4;

static ph4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  ph4 o = {{c0, c1, c2, c3}};
  return o;
}

static double u01(uint32_t a, uint32_t b) {
  return ((double)((((uint64_t)b << 32) | a) >> 11) + 0.5) * 0x1.0p-53;
}

static double d_from(uint64_t b) { double x; memcpy(&x, &b, 8); return x; }
static uint64_t d_bits(double x) { uint64_t b; memcpy(&b, &x, 8); return b; }

/* fdlibm e_log.c's algorithm, plain IEEE arithmetic (x finite, > 0) */
double oracle_det_log(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
               Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
               Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  uint64_t bits = d_bits(x);
  int32_t hx = (int32_t)(bits >> 32);
  int k = 0;
  if (hx < 0x00100000) {
    k -= 54;
    x *= 1.80143985094819840000e+16;
    bits = d_bits(x);
    hx = (int32_t)(bits >> 32);
  }
  k += (hx >> 20) - 1023;
  hx &= 0x000fffff;
  const int32_t i0 = (hx + 0x95f64) & 0x100000;
  x = d_from(((uint64_t)(uint32_t)(hx | (i0 ^ 0x3ff00000)) << 32) | (bits & 0xFFFFFFFFull));
  k += i0 >> 20;
  const double f = x - 1.0;
  const double dk = (double)k;
  if ((0x000fffff & (2 + hx)) < 3) {
    if (f == 0.0) return k == 0 ? 0.0 : dk * ln2_hi + dk * ln2_lo;
    const double R = f * f * (0.5 - 0.33333333333333333 * f);
    return k == 0 ? f - R : dk * ln2_hi - ((R - dk * ln2_lo) - f);
  }
  const double s = f / (2.0 + f);
  const double z = s * s;
  int32_t i = hx - 0x6147a;
  const double w = z * z;
  const int32_t j = 0x6b851 - hx;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  i |= j;
  const double R = t2 + t1;
  if (i > 0) {
    const double hfsq = 0.5 * f * f;
    return k == 0 ? f - (hfsq - s * (hfsq + R)) : dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
  }
  return k == 0 ? f - s * (f - R) : dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

static uint32_t gcd32(uint32_t a, uint32_t b) {
  while (b) { const uint32_t t = a % b; a = b; b = t; }
  return a;
}
static uint32_t coprime(uint32_t x, uint32_t m) {
  uint32_t a = (x % m) | 1u;
  if (a >= m) a = 1u;
  while (gcd32(a, m) != 1u) { a += 2u; if (a >= m) a = 1u; }
  return a;
}

static int kind_of(int r) { const int k5 = r % 5; return k5 == 1 || k5 == 4 ? 1 : (k5 == 2 ? 2 : 0); }
static double plant_p(int r) { const int k5 = r % 5; return k5 == 1 ? 0.5 : (k5 == 3 ? 0.8 : 0.9); }

static double value(uint32_t seed, uint32_t qlo, uint32_t qhi, int r, uint32_t i, int* pool) {
  const ph4 a = philox(i, (uint32_t)r, qlo, qhi, seed, 3);
  *pool = u01(a.x[0], a.x[1]) < 0.5;
  const double u0 = u01(a.x[2], a.x[3]);
  const ph4 b = philox(i, (uint32_t)r, qlo, qhi, seed, 4);
  const double u1 = u01(b.x[0], b.x[1]);
  const int kind = kind_of(r);
  if (kind == 1) return 5.0 - 6.0 * oracle_det_log(u0 * u1);
  const double u2 = u01(b.x[2], b.x[3]);
  const ph4 c = philox(i, (uint32_t)r, qlo, qhi, seed, 5);
  const double u3 = u01(c.x[0], c.x[1]), u4 = u01(c.x[2], c.x[3]);
  const ph4 d = philox(i, (uint32_t)r, qlo, qhi, seed, 6);
  const double u5 = u01(d.x[0], d.x[1]);
  const double us[6] = {u0, u1, u2, u3, u4, u5};
  double m1 = -1.0, m2 = -1.0;
  for (int t = 0; t < 6; ++t) {
    if (us[t] > m1) { m2 = m1; m1 = us[t]; }
    else if (us[t] > m2) { m2 = us[t]; }
  }
  return kind == 0 ? 0.5 + 0.4 * m2 : oracle_det_log(m2) - 1e-3;
}

static int cmp_desc(const void* x, const void* y) {
  const double a = *(const double*)x, b = *(const double*)y;
  return a < b ? 1 : (a > b ? -1 : 0);
}

/* lists [q_begin, q_begin + n_queries) x R of K entries; list_off[n*R+1], docid[n*R*K],
 * score[n*R*K]; qrel_off[n_qrel_q + 1] / qrel_doc: the judged documents (host arrays) */
int oracle_synth_runs_nq(int64_t q_begin, int64_t n_queries, int32_t R, int32_t K, uint64_t seed64,
                         const int64_t* qrel_off, const uint32_t* qrel_doc, int64_t n_qrel_q,
                         int64_t* list_off, uint32_t* docid, double* score) {
  const uint32_t seed = (uint32_t)seed64;
  const uint32_t P = 2u * (uint32_t)K, M = NQ_CORPUS - P;
  double* v = (double*)malloc(sizeof(double) * (size_t)(K > 0 ? K : 1));
  if (!v) return 1;
  for (int64_t l = 0; l < n_queries * R; ++l) {
    const int r = (int)(l % R);
    const uint64_t q = (uint64_t)(q_begin + l / R);
    const uint32_t qlo = (uint32_t)q, qhi = (uint32_t)(q >> 32);
    const ph4 hq = philox(qlo, qhi, 0u, 0u, seed, 1);
    const uint32_t a = (uint32_t)(((((uint64_t)hq.x[1]) << 32) | hq.x[0]) % (uint64_t)(M + 1u));
    const ph4 hl = philox(qlo, qhi, (uint32_t)r, 0u, seed, 2);
    const uint32_t Ap = coprime(hl.x[0], P), Bp = hl.x[1] % P;
    const uint32_t Ag = coprime(hl.x[2], M), Bg = hl.x[3] % M;
    uint32_t* ids = docid + l * (int64_t)K;
    uint32_t kp = 0u;
    for (uint32_t i = 0; i < (uint32_t)K; ++i) {
      int pool = 0;
      v[i] = value(seed, qlo, qhi, r, i, &pool);
      if (pool) {
        ids[i] = a + (uint32_t)(((uint64_t)Ap * kp + Bp) % P);
        ++kp;
      } else {
        const uint32_t g = (uint32_t)(((uint64_t)Ag * (i - kp) + Bg) % M);
        ids[i] = g < a ? g : g + P;
      }
    }
    qsort(v, (size_t)K, sizeof(double), cmp_desc);
    /* plant */
    if (n_qrel_q > 0) {
      const int64_t qq = (int64_t)(q % (uint64_t)n_qrel_q);
      int planted[16], np = 0;
      for (int64_t jj = qrel_off[qq]; jj < qrel_off[qq + 1] && jj - qrel_off[qq] < 16; ++jj) {
        const uint32_t d = qrel_doc[jj], jr = (uint32_t)(jj - qrel_off[qq]);
        const ph4 hp = philox(jr, (uint32_t)r, qlo, qhi, seed, 7);
        if (!(u01(hp.x[0], hp.x[1]) < plant_p(r))) continue;
        uint32_t t = 0u;
        while (t < 100000u) {
          const ph4 hg = philox(t, jr | ((uint32_t)r << 8), qlo, qhi, seed, 8);
          if (u01(hg.x[0], hg.x[1]) < 0.15) break;
          ++t;
        }
        int p = (int)t, moved = 1;
        while (moved && p < K) {
          moved = 0;
          for (int k = 0; k < np; ++k)
            if (planted[k] == p) { ++p; moved = 1; }
        }
        if (p >= K) continue;
        int found = -1;
        for (int i = 0; i < K; ++i)
          if (ids[i] == d) found = i;
        if (found >= 0) { ids[found] = ids[p]; ids[p] = d; }
        else ids[p] = d;
        planted[np++] = p;
      }
    }
    for (int i = 0; i < K; ++i) score[l * (int64_t)K + i] = v[i] + 1e-6 * (double)(K - 1 - i);
    list_off[l] = l * (int64_t)K;
  }
  list_off[n_queries * R] = n_queries * R * (int64_t)K;
  free(v);
  return 0;
}
