// qf_synth.hip — the benchmark's synthetic runs as SURVEY.md §8(d) specifies them
// (bench / tests only; qf_synth_runs_nq).
//
// Per query q and retriever r (BGE, BM25, BM25_MonoT5, BM25_TCT, Splade: sorted
// names, the learned models' order; r >= 5 repeats the five):
//  * K distinct docids: each position draws, with probability 0.5, from the query's
//    shared pool of P = 2K candidates (a block of P ids at a random base), otherwise
//    from the rest of the 2,681,468 NQ corpus ids (doc{n} -> n).  The k-th pool
//    position of a list takes pool id pi(k), the k-th other position id g(k), both
//    affine bijections drawn per list, so a list never repeats an id.
//  * scores: K iid draws sorted descending, plus 1e-6 * (K - 1 - rank) (strictly
//    decreasing in "%.6f"): BM25 and Splade Gamma(2, 6) + 5 (= 5 - 6 ln(u1 u2)),
//    BGE and BM25_TCT 0.5 + 0.4 Beta(5, 2), BM25_MonoT5 ln Beta(5, 2) - 0.001 (negative
//    after the tie-breaker) —
//    Beta(5, 2) as the second largest of six uniforms (an order statistic, no
//    transcendental), ln by det_log below.
//  * qrels: every judged document of the query (the committed NQ test qrels,
//    tests/golden/nq_qrels_test.tsv.gz; query q takes the judgments of q mod n) is
//    planted into list r with probability p_r = {0.9, 0.5, 0.9, 0.8, 0.9} at rank
//    ~ Geometric(0.15), in judgment order: a position already holding a planted
//    document moves it one further; a document already in the list is swapped there.
// Every draw is Philox4x32-10 keyed by (seed, stream) with the counter (position or
// step, retriever, query) — counter-based, so any query range (a rank's shard)
// regenerates independently, and oracle/synth_oracle.c regenerates it on the CPU bit
// for bit (the same operations: ln is fdlibm's algorithm in plain IEEE arithmetic,
// no transcendental library call, and -ffp-contract=off on both sides).
#include <hip/hip_runtime.h>
#include <hipcub/block/block_radix_sort.hpp>
#include <hipcub/block/block_scan.hpp>

#include "qf_common.h"
#include "qf_internal.h"

namespace qf {

constexpr uint32_t kNqCorpus = 2681468u;  // BEIR-NQ corpus size (doc0 .. doc2681467)

struct Philox4 {
  uint32_t x[4];
};
__device__ __forceinline__ Philox4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                          uint32_t k0, uint32_t k1) {
#pragma unroll
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
  return Philox4{{c0, c1, c2, c3}};
}
// (0, 1): 53 random bits, centred
__device__ __forceinline__ double synth_u01(uint32_t a, uint32_t b) {
  return ((double)((((uint64_t)b << 32) | a) >> 11) + 0.5) * 0x1.0p-53;
}

// ln x for finite x > 0 (fdlibm e_log.c's algorithm): plain IEEE +, -, *, / — the
// same bits on the CPU (oracle/synth_oracle.c) as here.
__device__ __forceinline__ double det_log(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
               Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
               Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  uint64_t bits = (uint64_t)__double_as_longlong(x);
  int32_t hx = (int32_t)(bits >> 32);
  int k = 0;
  if (hx < 0x00100000) {  // subnormal: scale up
    k -= 54;
    x *= 1.80143985094819840000e+16;
    bits = (uint64_t)__double_as_longlong(x);
    hx = (int32_t)(bits >> 32);
  }
  k += (hx >> 20) - 1023;
  hx &= 0x000fffff;
  const int32_t i0 = (hx + 0x95f64) & 0x100000;
  x = __longlong_as_double((int64_t)(((uint64_t)(uint32_t)(hx | (i0 ^ 0x3ff00000)) << 32) |
                                     (bits & 0xFFFFFFFFull)));
  k += i0 >> 20;
  const double f = x - 1.0;
  const double dk = (double)k;
  if ((0x000fffff & (2 + hx)) < 3) {  // |f| < 2^-20
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

__device__ __forceinline__ uint32_t synth_gcd(uint32_t a, uint32_t b) {
  while (b) {
    const uint32_t t = a % b;
    a = b;
    b = t;
  }
  return a;
}
// a multiplier coprime with m (odd start, + 2 until coprime; m > 2)
__device__ __forceinline__ uint32_t synth_coprime(uint32_t x, uint32_t m) {
  uint32_t a = (x % m) | 1u;
  if (a >= m) a = 1u;
  while (synth_gcd(a, m) != 1u) {
    a += 2u;
    if (a >= m) a = 1u;
  }
  return a;
}

// streams (the Philox key's second word)
enum : uint32_t { kStQuery = 1, kStList = 2, kStEntry = 3, kStPlant = 7, kStGeom = 8 };

// retriever kinds: 0 dense (0.5 + 0.4 Beta(5, 2)), 1 Gamma(2, 6) + 5, 2 ln Beta(5, 2)
__device__ __forceinline__ int synth_kind(int r) {
  const int k5 = r % 5;
  return k5 == 1 || k5 == 4 ? 1 : (k5 == 2 ? 2 : 0);
}
__device__ __forceinline__ double synth_plant_p(int r) {
  const int k5 = r % 5;
  return k5 == 1 ? 0.5 : (k5 == 3 ? 0.8 : 0.9);
}

// the unsorted score draw of position i of list (q, r)
__device__ __forceinline__ double synth_value(uint32_t seed, uint32_t qlo, uint32_t qhi, int r,
                                              uint32_t i, bool* pool) {
  const Philox4 a = philox(i, (uint32_t)r, qlo, qhi, seed, kStEntry);
  *pool = synth_u01(a.x[0], a.x[1]) < 0.5;
  const double u0 = synth_u01(a.x[2], a.x[3]);
  const Philox4 b = philox(i, (uint32_t)r, qlo, qhi, seed, kStEntry + 1);
  const double u1 = synth_u01(b.x[0], b.x[1]);
  const int kind = synth_kind(r);
  if (kind == 1) return 5.0 - 6.0 * det_log(u0 * u1);
  const double u2 = synth_u01(b.x[2], b.x[3]);
  const Philox4 c = philox(i, (uint32_t)r, qlo, qhi, seed, kStEntry + 2);
  const double u3 = synth_u01(c.x[0], c.x[1]), u4 = synth_u01(c.x[2], c.x[3]);
  const Philox4 d = philox(i, (uint32_t)r, qlo, qhi, seed, kStEntry + 3);
  const double u5 = synth_u01(d.x[0], d.x[1]);
  // Beta(5, 2): the 5th smallest (second largest) of six uniforms
  const double us[6] = {u0, u1, u2, u3, u4, u5};
  double m1 = -1.0, m2 = -1.0;
#pragma unroll
  for (int t = 0; t < 6; ++t) {
    if (us[t] > m1) {
      m2 = m1;
      m1 = us[t];
    } else if (us[t] > m2) {
      m2 = us[t];
    }
  }
  return kind == 0 ? 0.5 + 0.4 * m2 : det_log(m2) - 1e-3;  // (below 0 after the tie-breaker)
}

template <int ITEMS>
__global__ __launch_bounds__(256) void synth_nq_kernel(int64_t q_begin, int64_t n_queries, int32_t R,
                                                       int32_t K, uint32_t seed,
                                                       const int64_t* __restrict__ qrel_off,
                                                       const uint32_t* __restrict__ qrel_doc,
                                                       int64_t n_qrel_q,
                                                       int64_t* __restrict__ list_off,
                                                       uint32_t* __restrict__ docid,
                                                       double* __restrict__ score) {
  constexpr int BLOCK = 256, KMAX = BLOCK * ITEMS;
  using Sort = hipcub::BlockRadixSort<double, BLOCK, ITEMS>;
  using Scan = hipcub::BlockScan<uint32_t, BLOCK>;
  __shared__ union {
    typename Sort::TempStorage sort;
    typename Scan::TempStorage scan;
  } tmp;
  __shared__ uint32_t sid[KMAX];
  __shared__ int s_found, s_pos;
  __shared__ int planted[16];
  const int64_t l = block_id();
  const int tid = threadIdx.x;
  if (l == 0 && tid == 0) list_off[n_queries * R] = n_queries * R * (int64_t)K;
  if (l >= n_queries * R) return;
  if (tid == 0) list_off[l] = l * (int64_t)K;
  const int r = (int)(l % R);
  const uint64_t q = (uint64_t)(q_begin + l / R);
  const uint32_t qlo = (uint32_t)q, qhi = (uint32_t)(q >> 32);
  const uint32_t P = 2u * (uint32_t)K, M = kNqCorpus - P;
  // the query's pool block [a, a + P) and the list's two bijections
  const Philox4 hq = philox(qlo, qhi, 0u, 0u, seed, kStQuery);
  const uint32_t a = (uint32_t)(((((uint64_t)hq.x[1]) << 32) | hq.x[0]) % (uint64_t)(M + 1u));
  const Philox4 hl = philox(qlo, qhi, (uint32_t)r, 0u, seed, kStList);
  const uint32_t Ap = synth_coprime(hl.x[0], P), Bp = hl.x[1] % P;
  const uint32_t Ag = synth_coprime(hl.x[2], M), Bg = hl.x[3] % M;
  // positions 0..K-1 blocked over the threads (thread t: ITEMS t .. ITEMS t + ITEMS - 1)
  double v[ITEMS];
  uint32_t isp[ITEMS], npool = 0u;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = (uint32_t)(ITEMS * tid + j);
    bool pool = false;
    v[j] = -INFINITY;
    if (i < (uint32_t)K) v[j] = synth_value(seed, qlo, qhi, r, i, &pool);
    isp[j] = pool && i < (uint32_t)K;
    npool += isp[j];
  }
  uint32_t pre;  // pool positions before this thread's first
  Scan(tmp.scan).ExclusiveSum(npool, pre);
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = (uint32_t)(ITEMS * tid + j);
    if (i < (uint32_t)K) {
      const uint32_t kp = pre, kg = i - pre;  // this position's pool / other index
      uint32_t id;
      if (isp[j]) {
        id = a + (uint32_t)(((uint64_t)Ap * kp + Bp) % P);
      } else {
        const uint32_t g = (uint32_t)(((uint64_t)Ag * kg + Bg) % M);
        id = g < a ? g : g + P;
      }
      sid[i] = id;
      pre += isp[j];
    }
  }
  __syncthreads();  // (the scan's storage is reused by the sort)
  Sort(tmp.sort).SortDescendingBlockedToStriped(v);
  // ---- plant the query's judged documents ---------------------------------------------
  const int64_t qq = n_qrel_q > 0 ? (int64_t)(q % (uint64_t)n_qrel_q) : 0;
  const int64_t j0 = n_qrel_q > 0 ? qrel_off[qq] : 0, j1 = n_qrel_q > 0 ? qrel_off[qq + 1] : 0;
  int np = 0;  // planted positions so far (block-uniform)
  for (int64_t jj = j0; jj < j1 && jj - j0 < 16; ++jj) {
    const uint32_t d = qrel_doc[jj];
    const uint32_t jr = (uint32_t)(jj - j0);
    if (tid == 0) {
      int p = -1;
      const Philox4 hp = philox(jr, (uint32_t)r, qlo, qhi, seed, kStPlant);
      if (synth_u01(hp.x[0], hp.x[1]) < synth_plant_p(r)) {
        uint32_t t = 0u;  // Geometric(0.15) on {1, 2, ...}: failures before a success
        while (t < 100000u) {
          const Philox4 hg = philox(t, jr | ((uint32_t)r << 8), qlo, qhi, seed, kStGeom);
          if (synth_u01(hg.x[0], hg.x[1]) < 0.15) break;
          ++t;
        }
        p = (int)t;  // rank t + 1, position t
        bool moved = true;
        while (moved && p < K) {  // past the positions already planted
          moved = false;
          for (int k = 0; k < np; ++k)
            if (planted[k] == p) {
              ++p;
              moved = true;
            }
        }
        if (p >= K) p = -1;
      }
      s_pos = p;
      s_found = -1;
    }
    __syncthreads();
    const int p = s_pos;
    if (p >= 0) {  // uniform
      for (int i = tid; i < K; i += BLOCK)
        if (sid[i] == d) s_found = i;  // (ids are distinct: at most one writer)
      __syncthreads();
      if (tid == 0) {
        const int t = s_found;
        if (t >= 0) {  // already in the list: swap it to p
          sid[t] = sid[p];
          sid[p] = d;
        } else {
          sid[p] = d;
        }
        planted[np] = p;
      }
      ++np;
    }
    __syncthreads();
  }
  // ---- store: striped positions i = j * BLOCK + tid after the sort ------------------------
  const int64_t base = l * (int64_t)K;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int i = j * BLOCK + tid;
    if (i < K) {
      score[base + i] = v[j] + 1e-6 * (double)(K - 1 - i);
      docid[base + i] = sid[i];
    }
  }
}

hipError_t synth_nq_launch(int64_t q_begin, int64_t n_queries, int32_t R, int32_t K,
                           uint64_t seed, const int64_t* qrel_off, const uint32_t* qrel_doc,
                           int64_t n_qrel_q, int64_t* list_off, uint32_t* docid, double* score,
                           hipStream_t st) {
  const int64_t lists = n_queries * R;
  if (lists == 0) {
    hipLaunchKernelGGL((synth_nq_kernel<4>), dim3(1), dim3(256), 0, st, q_begin, (int64_t)0, R, K,
                       (uint32_t)seed, qrel_off, qrel_doc, n_qrel_q, list_off, docid, score);
    return hipGetLastError();
  }
  if (K <= 1024)
    hipLaunchKernelGGL((synth_nq_kernel<4>), grid_for(lists), dim3(256), 0, st, q_begin, n_queries,
                       R, K, (uint32_t)seed, qrel_off, qrel_doc, n_qrel_q, list_off, docid, score);
  else
    hipLaunchKernelGGL((synth_nq_kernel<16>), grid_for(lists), dim3(256), 0, st, q_begin,
                       n_queries, R, K, (uint32_t)seed, qrel_off, qrel_doc, n_qrel_q, list_off,
                       docid, score);
  return hipGetLastError();
}

}  // namespace qf
