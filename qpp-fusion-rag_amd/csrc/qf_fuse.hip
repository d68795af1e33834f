// qf_fuse.hip — multi-method rank fusion on gfx950: a join kernel + a fuse kernel.
//
// Replaces the per-row Python loops of src/fusion.py:
//   combsum / combmnz / rrf      (ranx fuse, src/fusion.py:170-230, 455-477)
//   weighted_combsum / _combmnz / weighted_rrf (src/fusion.py:237-380)
// and the per-query sort of write_runfile (src/fusion.py:480-492).
//
// join_kernel — one workgroup per query (N = Σ_r |list(q,r)| entries), all in LDS:
//   docids are inserted into an LDS hash table (open addressing, ds_cmpst); each
//   slot ORs in a retriever bit.  Lists are retriever-major with rows in file
//   order, so a document's first-seen entry (the reference's defaultdict
//   insertion order, src/fusion.py:264-279) is its entry in the lowest
//   retriever holding it.  Distinct documents are numbered u = 0..U-1 in
//   first-seen order (ballot + scan), and every entry is placed into its
//   document's contribution group, groups in u order, entries inside a group in
//   retriever order.  A retriever bit already set means a docid repeats inside
//   one list -> per-query error.  Then one thread per document adds its group's
//   contributions in retriever order — the reference's left-to-right sum, bit
//   for bit, no atomics — for every requested method at once, and writes the
//   unsorted fused scores to fused[slot][u].
// fuse_kernel — one workgroup per (query, method): reads fused[slot][0..U)
//   (coalesced) into registers in the sort's layout, stable-sorts by score
//   descending, ties in first-seen order (Python's stable sorted(),
//   src/fusion.py:475,488), and writes perm / fused back in place, coalesced.
#include <cstdlib>
#include <type_traits>

#include "../../include/qppfuse.h"
#include "qf_common.h"
#include "qf_internal.h"
#include "qf_lists.h"

namespace qf {

constexpr int kRMax = 16;    // runs per query in the LDS join (u16 retriever masks)
constexpr int kRMaxXl = 32;  // in the workspace kernel (u32 masks)
constexpr int kNMethods = 9;  // method bits QF_COMBSUM .. QF_WRRF_MUL
constexpr uint32_t kEmpty = 0xFFFFFFFFu;


// Score as stored: int32 micro-units (exact "%.6f" text) or double.
template <int KIND>
struct ScoreIn {
  using raw_t = double;
  static __device__ __forceinline__ raw_t raw(const void* p, int64_t i) {
    return ((const double*)p)[i];
  }
  static __device__ __forceinline__ double val(raw_t r) { return r; }
  static __device__ __forceinline__ double load(const void* p, int64_t i) { return raw(p, i); }
};
template <>
struct ScoreIn<1> {
  using raw_t = int32_t;
  static __device__ __forceinline__ raw_t raw(const void* p, int64_t i) {
    return ((const int32_t*)p)[i];
  }
  // m / 1e6 is the nearest double to the "%.6f" text, i.e. pandas' parse
  // (correctly rounded without a division: qf_common.h micro_to_f64).
  static __device__ __forceinline__ double val(raw_t r) { return micro_to_f64(r); }
  static __device__ __forceinline__ double load(const void* p, int64_t i) { return val(raw(p, i)); }
};

// The weight of list (q, r): p.weights, or (qf_fuse_qpp) the .qpp round trip of the
// raw predictors normalised with the column statistics — qpp_normalize_kernel's
// w_out bit for bit (src/qpp.py:356-372, src/fusion.py:150-158), computed by the
// join's per-list threads while the entries' loads are in flight.
__device__ __forceinline__ double list_weight(const FuseParams& p, int64_t q, int r,
                                              bool present) {
  if (!p.qpp_raw) return p.weights ? p.weights[q * p.R + r] : 1.0;
  const int64_t l = q * p.R + r;
  const int mode = p.qpp_mode;
  const double* x = p.qpp_raw + l * kQppCols;
  const double* m0 = p.qpp_stats + (int64_t)r * kQppCols;
  const double* m1 = p.qpp_stats + ((int64_t)p.R + r) * kQppCols;
  auto back = [&](int c) {
    return micro_back(round6(qpp_norm_value(x[c], mode != 0 ? m0[c] : 0.0,
                                            mode != 0 ? m1[c] : 0.0, mode, present)));
  };
  if (p.qpp_index >= 0) return back(p.qpp_index);
  double wsum = 0.0;  // Python sum(): left to right
#pragma unroll
  for (int c = 0; c < kQppCols; ++c) wsum += back(c);
  return wsum / (double)kQppCols;
}

// ---- block-level helpers ------------------------------------------------------

// The value of lane + 1 (DPP wave_shl:1, one VALU per dword; lane 63 gets its own
// old value — callers treat lane 63 separately).
__device__ __forceinline__ int32_t shl1_lane(int32_t v) {
  return __builtin_amdgcn_update_dpp(v, v, 0x130, 0xf, 0xf, false);
}
__device__ __forceinline__ double shl1_lane(double v) {
  const int64_t b = __double_as_longlong(v);
  const int32_t lo = __builtin_amdgcn_update_dpp((int32_t)b, (int32_t)b, 0x130, 0xf, 0xf, false);
  const int32_t hi = __builtin_amdgcn_update_dpp((int32_t)(b >> 32), (int32_t)(b >> 32), 0x130,
                                                 0xf, 0xf, false);
  return __longlong_as_double(((int64_t)hi << 32) | (uint32_t)lo);
}

// Raw v_min_f64 / v_max_f64, without fmin / fmax's NaN canonicalisation (three
// more instructions per call): the callers flag NaNs themselves and discard the
// range when one is present.
__device__ __forceinline__ double raw_min_f64(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double raw_max_f64(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// min(a, -b) in one instruction (the negation is a source modifier)
__device__ __forceinline__ double raw_min_neg_f64(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, -%2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// MIN / MAX of a 64-bit key over the block (s_min / s_max pre-initialised; a
// barrier must separate this call from reading the result).
__device__ __forceinline__ void block_min_max(uint64_t kmn, uint64_t kmx,
                                              unsigned long long* s_min,
                                              unsigned long long* s_max, int lane) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    kmn = min(kmn, (uint64_t)__shfl_xor((unsigned long long)kmn, d, 64));
    kmx = max(kmx, (uint64_t)__shfl_xor((unsigned long long)kmx, d, 64));
  }
  if (lane == 0) {
    atomicMin(s_min, (unsigned long long)kmn);
    atomicMax(s_max, (unsigned long long)kmx);
  }
}

// ---- the per-(query, method) sort -------------------------------------------
//
// Items are 32-bit words, held in registers wave-major (item i = (wid*rows +
// j)*64 + lane) and scattered through LDS between passes:
//   bits 14..31  window key: the kWindow most significant bits of (wkey - wmin),
//                a non-decreasing function of key = ~orderable(score)
//                (ascending key == descending score), see sort_one
//   bits  0..13  u, the document's first-seen index
// The full key of an item is re-derived from fused[u] (the unsorted scores in
// HBM/L2), which only the rare fix-up and the output need.
constexpr int kDigit = 9;                // bits per LSD pass
constexpr int kBuckets = 1 << kDigit;    // counters per wave, 16 bits each
constexpr int kUBits = 14;
constexpr uint32_t kUMask = (1u << kUBits) - 1u;
template <int ITEMS, int WAVES>
struct SortCtx {
  uint32_t* hist;      // [WAVES][kBuckets] u16 counters, two per word
  uint32_t* sitem;     // [UMAX]
  const double* sval;  // fused[slot] of the query: the unsorted scores by u
  uint32_t* wtot;      // [WAVES] scan carries
  int* flag;           // [2]: fix-up status, listed runs
  uint64_t kmin;
  int U, rows, lane, wid, tid;
};

template <int ITEMS, int WAVES>
__device__ __forceinline__ uint64_t full_key(const SortCtx<ITEMS, WAVES>& sx, uint32_t item) {
  return ~f64_asc_key(sx.sval[item & kUMask]);
}

// The lanes of the wave (active ones) whose kDigit-bit digit equals this lane's:
// one ballot per digit bit; a lane disagrees with the lanes set in ballot ^ t (t =
// its own bit as 0 / all ones, one v_bfe_i32), whose union is accumulated — five
// VALU per bit (bfe, compare, two xor, or) where the select form took nine.
__device__ __forceinline__ uint64_t match_digit(uint32_t d, bool active) {
  uint32_t dl = 0u, dh = 0u;  // lanes whose digit differs from this lane's
#pragma unroll
  for (int b = 0; b < kDigit; ++b) {
    uint32_t t = (uint32_t)__builtin_amdgcn_sbfe((int)d, (uint32_t)b, 1u);
    asm("" : "+v"(t));  // compare t itself (not a shifted copy of d: one op more)
    const uint64_t bb = ballot(t != 0u);
    dl |= (uint32_t)bb ^ t;
    dh |= (uint32_t)(bb >> 32) ^ t;
  }
  return ballot(active) & ~(((uint64_t)dh << 32) | dl);
}

// One stable counting-scatter pass on a kDigit-bit digit of the items.  Within a
// wave every item's rank among the wave's items with its digit, in item order, is
// built from orders the ISA fixes: inside a row, the lanes with its digit below it
// (a ballot match, match_digit); across rows, the row's one returning LDS atomic
// per digit — issued by the digit's lowest lane, adding the row's count — since a
// wave's LDS instructions complete in program order.  No result depends on the
// order in which one instruction's same-address atomics are applied.  The (wave,
// digit) offsets are one block-wide exclusive scan in [digit][wave] order.  Leaves
// the scattered sequence in sitem; `readback` reloads the registers.
template <int ITEMS, int WAVES>
__device__ __forceinline__ void count_scatter(const SortCtx<ITEMS, WAVES>& sx,
                                              uint32_t (&item)[ITEMS], int sh, bool readback) {
  const int lane = sx.lane, wid = sx.wid;
  int rp = sx.rows;
  asm volatile("" : "+s"(rp));
  // digit = bits sh..sh+8 of the window key
  auto digit = [sh](uint32_t it) -> uint32_t {
    return __builtin_amdgcn_ubfe(it, (uint32_t)(kUBits + sh), (uint32_t)kDigit);
  };
  // hist is [wave][digit] u16 counters (digit d: word d >> 1, half d & 1; a
  // wave's leaders hit distinct banks); counts and offsets stay below 2^16
  uint32_t* hist = sx.hist;
  uint16_t* hist16 = (uint16_t*)sx.hist;
  for (int k = lane; k < kBuckets / 2; k += 64) hist[wid * (kBuckets / 2) + k] = 0u;
  // Rank of every item among its wave's items with the same digit, in item
  // order (see above).  Round 3 took it from one ds_add_rtn per item, which is
  // stable only because gfx950 happens to apply one instruction's same-address
  // atomics in lane order (tools/lds_atomic_order.hip measured it; the ISA does
  // not promise it): the match costs ~60 more VALU per row, on the paths that use
  // this sort (small unions, the bucket sort's fallback pass, probFuse).
  uint32_t rank_in[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    rank_in[j] = 0u;
    if (j < rp) {  // wave-uniform
      const int i = (wid * rp + j) * 64 + lane;
      const bool act = i < sx.U;
      const uint32_t d = act ? digit(item[j]) : 0u;
      const uint64_t same = match_digit(d, act);
      const uint32_t below = mbcnt(same);  // same-digit lanes before this one
      const uint32_t hs = (d & 1u) * 16u;
      uint32_t old = 0u;
      if (act && below == 0u)  // the digit's lowest lane adds the row's count
        old = atomicAdd(&hist[wid * (kBuckets / 2) + (d >> 1)],
                        (uint32_t)__popcll(same) << hs);
      const int leader = same ? __ffsll((unsigned long long)same) - 1 : lane;
      old = (uint32_t)__builtin_amdgcn_ds_bpermute(leader << 2, (int)old);
      if (act) rank_in[j] = ((old >> hs) & 0xFFFFu) + below;
    }
  }
  __syncthreads();
  // block-wide exclusive scan of the kBuckets*WAVES counters in [digit][wave]
  // order, kPer per thread (16-bit loads and stores: no word is shared)
  {
    constexpr int kPer = kBuckets / 64;
    uint32_t v[kPer], t = 0u;
#pragma unroll
    for (int c = 0; c < kPer; ++c) {
      const int f = kPer * sx.tid + c;
      v[c] = hist16[(f % WAVES) * kBuckets + f / WAVES];
      t += v[c];
    }
    const uint32_t incl = wave_incl_scan_dpp(t);
    if (lane == 63) sx.wtot[wid] = incl;
    __syncthreads();
    uint32_t ex = incl - t;
#pragma unroll
    for (int w = 0; w < WAVES; ++w)
      if (w < wid) ex += sx.wtot[w];
#pragma unroll
    for (int c = 0; c < kPer; ++c) {
      const int f = kPer * sx.tid + c;
      hist16[(f % WAVES) * kBuckets + f / WAVES] = (uint16_t)ex;
      ex += v[c];
    }
  }
  __syncthreads();
  asm volatile("" : "+s"(rp));
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int i = (wid * rp + j) * 64 + lane;
    if (j < rp && i < sx.U)
      sx.sitem[hist16[wid * kBuckets + digit(item[j])] + rank_in[j]] = item[j];
  }
  __syncthreads();
  if (readback) {
    asm volatile("" : "+s"(rp));
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const int i = (wid * rp + j) * 64 + lane;
      if (j < rp && i < sx.U) item[j] = sx.sitem[i];
    }
  }
}

// Lane l gets lane l-1's value (DPP wave_shr:1; lane 0 gets its own back).
__device__ __forceinline__ uint32_t wave_up1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x138, 0xf, 0xf, false);
}

// Stable sort of the items by full key ascending (scores descending; ties keep
// input = first-seen order), given the window width nb (<= kWindow):
//  1. LSD counting passes over the window key;
//  2. unless the window is exact (every bit of the full key): inside a run of
//     items with equal window keys an item is "bad" when its predecessor has a
//     larger full key.  No bad item anywhere (the usual case; long runs of equal
//     keys are never bad): sorted.  Otherwise the run of each first bad item is
//     put in full-key order by a stable insertion sort run by one thread.
// A run longer than kRunMax that needs fixing sends the block on with LSD passes
// over every bit of (full key - kmin) (hb_full bits) from bit 0: started from
// the order of step 1 (equal keys still first-seen) they give the same stable
// result.
constexpr int kRunMax = 64;
constexpr int kWindow = 2 * kDigit;  // bits sorted by LSD passes (2 passes of 9)
static_assert(kWindow + kUBits <= 32, "items are 32-bit");

template <int ITEMS, int WAVES>
__device__ void sort_desc(const SortCtx<ITEMS, WAVES>& sx, uint32_t (&item)[ITEMS], int nb,
                          bool exact, int hb_full) {
  int sh = 0;
  bool fallback = false;
  if (sx.tid == 0) { sx.flag[0] = 0; sx.flag[1] = 0; }  // ordered by count_scatter's barriers
  constexpr int kListCap = (kBuckets / 2) * WAVES;     // run starts, kept in hist
#pragma unroll 1
  while (true) {
    if (fallback) {  // this pass's digit of the full key becomes the window key
      int rp = sx.rows;
      asm volatile("" : "+s"(rp));
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        const int i = (sx.wid * rp + j) * 64 + sx.lane;
        if (j < rp && i < sx.U)
          item[j] = ((uint32_t)(((full_key(sx, item[j]) - sx.kmin) >> sh) &
                                (uint64_t)(kBuckets - 1)) << kUBits) | (item[j] & kUMask);
      }
    }
    count_scatter(sx, item, fallback ? 0 : sh, true);
    sh += kDigit;
    if (sh < (fallback ? hb_full : nb)) continue;
    if (fallback || exact) return;
    // -- A: find the runs to fix (read-only) ----------------------------------------
    // First every row's predecessor window and, where the windows tie, both scores
    // are loaded (all rows' loads in flight at once), then compared: one memory
    // latency per wave, not one per row.
    {
      int rp = sx.rows;
      asm volatile("" : "+s"(rp));
      bool any = false;
      double vk[ITEMS], vp[ITEMS];
      uint32_t tie = 0u;
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        const int i = (sx.wid * rp + j) * 64 + sx.lane;
        const uint32_t wk = item[j] >> kUBits;
        uint32_t wp = wave_up1(wk);
        vk[j] = vp[j] = 0.0;
        if (j < rp && i < sx.U && i > 0) {
          const uint32_t ip = sx.sitem[i - 1];
          if (sx.lane == 0) wp = ip >> kUBits;
          if (wp == wk) {  // same window as the predecessor: fetch both scores
            tie |= 1u << j;
            vk[j] = sx.sval[item[j] & kUMask];
            vp[j] = sx.sval[ip & kUMask];
          }
        }
      }
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        if (!((tie >> j) & 1u)) continue;
        const int i = (sx.wid * rp + j) * 64 + sx.lane;
        const uint32_t wk = item[j] >> kUBits;
        const uint64_t k = ~f64_asc_key(vk[j]), kp = ~f64_asc_key(vp[j]);
        if (kp > k) {  // bad: walk back to the run start
          any = true;
          int st = i - 1;
          uint64_t kc = kp;
          bool first = true;
          while (st > 0) {
            const uint32_t iq = sx.sitem[st - 1];
            if ((iq >> kUBits) != wk) break;
            const uint64_t kq = full_key(sx, iq);
            if (kq > kc) { first = false; break; }  // an earlier bad item owns the run
            kc = kq;
            --st;
            if (i - st > kRunMax) break;
          }
          if (first) {
            if (i - st > kRunMax) {
              atomicOr(&sx.flag[0], 1);
            } else {
              const int slot = atomicAdd(&sx.flag[1], 1);
              if (slot < kListCap) sx.hist[slot] = (uint32_t)st;
              else atomicOr(&sx.flag[0], 1);
            }
          }
        }
      }
      if (any) atomicOr(&sx.flag[0], 2);
    }
    __syncthreads();
    const int f = sx.flag[0];  // block-uniform
    if (f == 0) return;        // no bad item: already in full-key order
    if (!(f & 1)) {
      // -- B: stable insertion sort of each listed run on the full key -------------
      const int nr = sx.flag[1];
      for (int t = sx.tid; t < nr; t += WAVES * 64) {
        const int i = (int)sx.hist[t];
        const uint32_t wk = sx.sitem[i] >> kUBits;
        int L = 1;
        while (i + L < sx.U && (sx.sitem[i + L] >> kUBits) == wk && L <= kRunMax) ++L;
        if (L > kRunMax) { atomicOr(&sx.flag[0], 1); continue; }
        for (int a = i + 1; a < i + L; ++a) {
          const uint32_t ia = sx.sitem[a];
          const uint64_t ka = full_key(sx, ia);
          int b = a - 1;
          while (b >= i && full_key(sx, sx.sitem[b]) > ka) {
            sx.sitem[b + 1] = sx.sitem[b];
            --b;
          }
          if (b + 1 != a) sx.sitem[b + 1] = ia;
        }
      }
      __syncthreads();
    }
    if (sx.flag[0] & 1) {  // a run too long: finish with full LSD passes
      fallback = true;
      sh = 0;
      continue;            // registers still hold the step-1 order
    }
    int rp = sx.rows;
    asm volatile("" : "+s"(rp));
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const int i = (sx.wid * rp + j) * 64 + sx.lane;
      if (j < rp && i < sx.U) item[j] = sx.sitem[i];
    }
    return;
  }
}

// Sorted items -> perm (u of rank i).  The scores stay where the join left them,
// by u: the ranked list is fused[perm[i]] (include/qppfuse.h).
template <int ITEMS, int WAVES>
__device__ __forceinline__ void write_out(const SortCtx<ITEMS, WAVES>& sx,
                                          const uint32_t (&item)[ITEMS], const FuseParams& p,
                                          int64_t po) {
  int ro = sx.rows;
  asm volatile("" : "+s"(ro));
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int i = (sx.wid * ro + j) * 64 + sx.lane;
    // final outputs, not re-read by the device: non-temporal, so they do not evict
    // the unsorted scores other workgroups are about to gather
    if (j < ro && i < sx.U) perm_put(p, po + i, item[j] & kUMask);
  }
}

// ---- one document's fused scores --------------------------------------------
// learned_fusion's row term and groupby-sum step (src/fusion.py:436-441): pandas
// Kahan summation in the column's dtype.  LightGBM weights are float64; FusionMLP's
// are float32, and under numpy 2 row["score"] * np.float32 is a float32 product, so
// its column is float32 (summed in float32) unless some run is unknown to the
// model (1.0 / n_retrievers: float64 products, a float64 column).
__device__ __forceinline__ void learned_add(const FuseParams& p, double s, double w, int r,
                                            double& a, double& c) {
  if (p.learned_f32 == 0u) {
    const double y = s * w - c;
    const double t = a + y;
    c = (t - a) - y;
    if (c != c) c = 0.0;  // +-inf contributions (pandas GH#53606)
    a = t;
    return;
  }
  const double v = ((p.learned_f32 >> r) & 1u) ? (double)((float)s * (float)w) : s * w;
  if (p.learned_sum_f32) {
    const float af = (float)a, cf = (float)c;
    const float y = (float)v - cf;
    const float t = af + y;
    float cn = (t - af) - y;
    if (cn != cn) cn = 0.0f;
    c = cn;
    a = t;
  } else {
    const double y = v - c;
    const double t = a + y;
    c = (t - a) - y;
    if (c != c) c = 0.0;
    a = t;
  }
}

// Per-list constants of one query (ranx min-max end points, QPP weights, offsets).
struct ListConsts {
  const int64_t* off;  // [R + 1] absolute list offsets
  const double* w;     // [R] weights (1.0 without)
  const double* mn;    // [R] list minimum (ranx min-max)
  const double* den;   // [R] max - min
  const double* rden;  // [R] 1 / (max - min)
};
// Adds a document's contributions in retriever order — the reference's
// left-to-right sums, bit for bit — for every requested method at once, and
// stores them unsorted at fused[slot][at]: the workspace join of very large
// queries.  The LDS join spells the same sums out inline (through this helper
// the C2 join spills 32 more bytes per thread; tests/test_gpu_fusion.py checks
// both paths against the oracle).
struct DocSums {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a5 = 0.0, a6 = 0.0, c6 = 0.0, a7 = 0.0, a8 = 0.0;
  __device__ __forceinline__ void add(const FuseParams& p, int methods, const ListConsts& lc,
                                      double s, int r, int pos) {
    if (methods & (QF_COMBSUM | QF_COMBMNZ)) {  // ranx min-max normalised score
      const double den = lc.den[r], mn = lc.mn[r];
      // A .norm.res list is already [0, 1] (min 0.000000, max 1.000000), where
      // (s - 0.0) / 1.0 == s bit for bit (-0.0 included): skip the division.
      double x = 0.0;
      if (den > 0.0) {
        const double d = s - mn;
        x = (den == 1.0 && mn == 0.0) ? s
            : (den >= 0x1p-900 && den <= 0x1p900 && d >= 0x1p-900 && d <= 0x1p900)
                ? div_by_recip(d, den, lc.rden[r])
                : d / den;
      }
      a0 += x;
    }
    if (methods & QF_RRF) a1 += recip_int(p.rrf_k + pos + 1);  // ranx rrf: rank = position
    if (methods & (QF_WCOMBSUM | QF_WCOMBMNZ)) a2 += lc.w[r] * s;  // src/fusion.py:273
    if (methods & QF_WRRF) {                                       // src/fusion.py:374
      const int rk = p.rank ? p.rank[lc.off[r] + pos] : pos + 1;
      a5 += div_int(lc.w[r], p.rrf_k + rk);
    }
    if (methods & (QF_PROBFUSE | QF_WRRF_MUL)) {
      const int rk = p.rank ? p.rank[lc.off[r] + pos] : pos + 1;  // int(row["rank"])
      if (methods & QF_PROBFUSE) {  // ProbFuse.py:30-39,172-179
        // ceil(rank * x / L) in integers (exact: the float quotient of two
        // integers below 2^26 is never rounded onto an integer), clipped to [1, x]
        const int64_t pp = rk > 0 ? rk : 1;
        int64_t k = (pp * p.n_seg + p.seg_len - 1) / p.seg_len;
        k = k < 1 ? 1 : (k > p.n_seg ? p.n_seg : k);
        a7 += div_int(p.seg_prob[r * p.n_seg + (int)k - 1], (int)k);
      }
      if (methods & QF_WRRF_MUL)  // QPPrrf_argmax.py:71: weight * (1.0 / (k + rank))
        a8 += lc.w[r] * recip_int(p.rrf_k + rk);
    }
    if (methods & QF_LEARNED) learned_add(p, s, lc.w[r], r, a6, c6);  // src/fusion.py:436-446
  }
  // cnt: the document's list count (CombMNZ: sum x count, src/fusion.py:327).
  // Output slot of method bit t: the requested methods below it (scalar popcounts).
  __device__ __forceinline__ void store(const FuseParams& p, int methods, double cnt,
                                        int64_t at) const {
    double* out = p.fused + at;
    const int64_t st = p.out_stride;
    auto slot = [&](int t) -> int64_t { return __popc((unsigned)methods & ((1u << t) - 1u)); };
    if (methods & QF_COMBSUM) out[slot(0) * st] = a0;
    if (methods & QF_COMBMNZ) out[slot(1) * st] = a0 * cnt;
    if (methods & QF_RRF) out[slot(2) * st] = a1;
    if (methods & QF_WCOMBSUM) out[slot(3) * st] = a2;
    if (methods & QF_WCOMBMNZ) out[slot(4) * st] = a2 * cnt;
    if (methods & QF_WRRF) out[slot(5) * st] = a5;
    if (methods & QF_LEARNED) out[slot(6) * st] = a6;
    if (methods & QF_PROBFUSE) out[slot(7) * st] = a7;
    if (methods & QF_WRRF_MUL) out[slot(8) * st] = a8;
  }
};

// ============================================================================
// join_kernel
// ============================================================================
template <int BLOCK, int ITEMS, int TB, int MINW = 1>
struct JoinCfg {
  static constexpr int kBlock = BLOCK, kItems = ITEMS, kWaves = BLOCK / 64, kMinWaves = MINW;
  static constexpr int kNMax = BLOCK * ITEMS, kTS = 1 << TB, kTB = TB;
  static_assert(kTS >= kNMax, "hash table must hold every entry");
  static_assert(kNMax <= 65535, "u / group offsets are uint16");
};

// LDS of the join: the hash table — tkey u32 [TS], retriever masks u16 [TS]
// (packed two per word) — later overlaid by the grouped contributions: scores
// as stored (int32 micro-units or f64) [NMAX], position | retriever u32 [NMAX],
// group starts u16 [NMAX].  Micro-unit scores keep JoinM at 50 KB: 3 per CU.
template <class C, int KIND>
struct JoinLds {
  using raw_t = typename ScoreIn<KIND>::raw_t;
  static constexpr int kTable = 6 * C::kTS;
  static constexpr int kGscOff = 0;
  static constexpr int kGprOff = (int)sizeof(raw_t) * C::kNMax;
  static constexpr int kGoOff = kGprOff + 4 * C::kNMax;
  static constexpr int kGroups = kGoOff + 2 * C::kNMax;
  static constexpr int kBytes = ((kTable > kGroups ? kTable : kGroups) + 15) & ~15;
  static_assert(kBytes <= 160 * 1024, "LDS budget");
};

// Shared memory of the join: the table / groups area (Extra: bytes the fused
// join + sort kernel reuses it for) and the per-query constants.
template <class C, int KIND, int EXTRA = 0>
struct JoinShared {
  using L = JoinLds<C, KIND>;
  static constexpr int kBytes = L::kBytes > EXTRA ? L::kBytes : EXTRA;
  __attribute__((aligned(16))) unsigned char smem[kBytes];
  int64_t off[kRMax + 1];
  int offr[kRMax + 1];  // off - off[0]: the join's 32-bit list boundaries
  double w[kRMax], mn[kRMax], den[kRMax], rden[kRMax];
  int cnt[C::kItems * C::kWaves], gof[C::kItems * C::kWaves];
  // lane 0's score of every (row, wave): lane 63's successor for the sort check
  typename ScoreIn<KIND>::raw_t first[C::kItems * C::kWaves + 1];
  double wres[12][C::kWaves];  // pair_info: every wave's reduced slot ranges
  int U, status;
  int slow;  // bit 0: a non-empty list is not [0, 1]-normalised; bit 1: a weight needs IEEE division
};

// The join proper, phases 1-3 (see the file header): loads, LDS hash join with the
// order / duplicate checks, first-seen numbering (union_docid written) and the
// contribution groups left in LDS (gsc / gpr / ugo of JoinLds).  Returns N, or -1
// when the query exceeds the configuration (union_count already written);
// sh.U / sh.status are set (block-uniform after the final barrier).
template <class C, int KIND, int EXTRA>
__device__ __forceinline__ int join_groups(const FuseParams& p, JoinShared<C, KIND, EXTRA>& sh,
                                           int64_t q) {
  constexpr int BLOCK = C::kBlock, ITEMS = C::kItems, WAVES = C::kWaves;
  constexpr int NMAX = C::kNMax, TS = C::kTS;
  using L = JoinLds<C, KIND>;
  using raw_t = typename L::raw_t;
  unsigned char* smem = sh.smem;
  uint32_t* tkey = (uint32_t*)smem;
  uint32_t* tmask2 = (uint32_t*)(smem + 4 * TS);  // two u16 masks per word
  auto mask_of = [&](uint32_t slot) -> uint32_t {
    return (tmask2[slot >> 1] >> ((slot & 1u) * 16u)) & 0xFFFFu;
  };
  const int tid = threadIdx.x, lane = tid & 63,
            wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: SGPR
  const int R = p.R;
  if (tid <= R) sh.off[tid] = p.list_off[q * R + tid];
  if (tid == 0) {
    sh.status = 0;
    sh.slow = 0;
  }
  __syncthreads();
  const int64_t base = sh.off[0];
  const int64_t N64 = sh.off[R] - base;
  // qf_fuse_qpp_micro: the .qpp values of this query's lists — every column of every
  // list, src/qpp.py:356-372 + the "%.6f" of :333, qpp_normalize_kernel's micro_out —
  // one value per thread past wave 0 (whose per-list threads compute the weights),
  // issued after the entries' loads (its loads' wait then overlaps theirs: issued
  // before them, it cost the join ~8 us on C2); a query the workspace join takes
  // gets its values before the early return
  auto qpp_micro = [&]() __attribute__((always_inline)) {
    const int t2 = BLOCK > 64 ? (tid + BLOCK - 64) % BLOCK : tid;
    for (int i = t2; i < R * kQppCols; i += BLOCK) {
      const int r = i / kQppCols, c = i - r * kQppCols;
      const int64_t l = q * R + r;
      const bool present = sh.off[r + 1] > sh.off[r];
      const int mode = p.qpp_mode;
      const double m0 = mode != 0 ? p.qpp_stats[r * kQppCols + c] : 0.0;
      const double m1 = mode != 0 ? p.qpp_stats[(R + r) * kQppCols + c] : 0.0;
      p.qpp_micro[l * kQppCols + c] =
          round6(qpp_norm_value(p.qpp_raw[l * kQppCols + c], m0, m1, mode, present));
    }
  };
  if (N64 > NMAX) {  // uniform
    if (p.qpp_micro) qpp_micro();
    if (tid == 0) p.union_count[q] = QF_QSTATUS_TOOBIG;
    return -1;
  }
  const int N = (int)N64;
  if (tid <= R) sh.offr[tid] = (int)(sh.off[tid] - base);  // read after the next barrier
  uint32_t dk[ITEMS];
  raw_t sc[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {  // all loads in flight before the first use
    const int e = j * BLOCK + tid;
    // (plain loads: non-temporal ones measured 122-124 -> 128-129 us, round 4)
    dk[j] = e < N ? p.docid[base + e] : kEmpty;
    sc[j] = e < N ? ScoreIn<KIND>::raw(p.score, base + e) : (raw_t)0;
  }
  // the per-list constants after the entries' loads are issued: wave 0's waits on
  // them then overlap the entries' latency instead of delaying its loads
  if (tid < R) {
    const int64_t a = sh.off[tid], b = sh.off[tid + 1];
    // ranx min-max (norm="min-max", the fuse() default); lists are sorted
    // descending (checked below), so max / min are the end points.  The three
    // loads are issued together (one latency)
    const double wv = list_weight(p, q, tid, b > a);
    double mx = 0.0, mn = 0.0;
    if (b > a) {
      mx = ScoreIn<KIND>::load(p.score, a);
      mn = ScoreIn<KIND>::load(p.score, b - 1);
    }
    sh.w[tid] = wv;
    sh.mn[tid] = mn;
    sh.den[tid] = ranx_den(mx, mn);
    sh.rden[tid] = 1.0 / sh.den[tid];  // one IEEE division per list (div_by_recip)
    // block-uniform fast paths of the sums: every list already [0, 1] (a .norm.res
    // list: x = s), every weight in div_int's division-free range
    const double aw = fabs(sh.w[tid]);
    const int slow = ((b > a && !(mx == 1.0 && mn == 0.0)) ? 1 : 0) |
                     ((aw > 0x1p-900 && aw < 0x1p900) ? 0 : 2);
    if (slow) atomicOr(&sh.slow, slow);
  }
  if (p.qpp_micro) qpp_micro();  // uniform
  for (int i = tid * 4; i < TS; i += BLOCK * 4)
    *(uint4*)&tkey[i] = make_uint4(kEmpty, kEmpty, kEmpty, kEmpty);
  for (int i = tid * 4; i < TS / 2; i += BLOCK * 4)
    *(uint4*)&tmask2[i] = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();
  QF_STOP(11, [&] { uint32_t a = 0u; for (int j = 0; j < ITEMS; ++j) a += dk[j] + (uint32_t)sc[j]; return a; },
          if (_qf_acc == 12345u || threadIdx.x == 0) p.union_count[q] = 0; return -1;);
  // ---- insert: entry e = j*BLOCK + tid of list r(e) --------------------------
  int status = 0;
  uint32_t rj[ITEMS];
  uint32_t defer = 0u;  // lane 63: rows whose successor (lane 0 of the next wave) is checked below
  const bool ranx = p.methods & (QF_COMBSUM | QF_COMBMNZ | QF_RRF);
  int r = 0;  // entry e's list; e grows with j, so the search resumes where it stopped
  // the end of list r (32-bit boundaries relative to the query's base), carried
  // from row to row: a row reads a boundary only when it crosses one
  int end = sh.offr[1];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int e = j * BLOCK + tid;
    // entry e + 1 (lane 63: garbage, checked below from LDS): DPP wave_shl:1
    const raw_t nxt = shl1_lane(sc[j]);
    rj[j] = 0u;
    if (lane == 0 && e < N) sh.first[j * WAVES + wid] = sc[j];
    if (e < N) {
      const uint32_t d = dk[j];
      if (d == kEmpty) status = QF_QSTATUS_BADDOC;
      while (e >= end) end = sh.offr[++r + 1];
      rj[j] = (uint32_t)r;
      // triangular probes (h + 1, + 2, + 3 ...: every slot of the power-of-two table):
      // no primary clustering.  A wave's row waits for its longest chain; on SURVEY
      // §8(d)'s unions (table load ~0.5) linear probes made the insert 55 of the
      // join's ~190 us, these 16 us less (round 5)
      uint32_t h = (d * 0x9E3779B1u) >> (32 - C::kTB), step = 1u;
      while (true) {
        const uint32_t prev = atomicCAS(&tkey[h], kEmpty, d);
        if (prev == kEmpty || prev == d) break;
        h = (h + step++) & (TS - 1);
      }
      const uint32_t hs = (h & 1u) * 16u;
      const uint32_t old = atomicOr(&tmask2[h >> 1], (1u << r) << hs);
      if ((old >> (hs + r)) & 1u) status = QF_QSTATUS_DUPDOC;
      dk[j] = h;  // keep the slot
      // preconditions of the ranx methods / W-RRF (checked once, here)
      const int64_t g = base + e;
      if (e + 1 < end) {
        if (ranx) {
          // raw compare: m / 1e6 is strictly increasing in the micro-units m.
          // Lane 63's successor is lane 0 of the next wave: compared after the
          // barrier from LDS (a global load here stalled every row)
          if (lane == 63) defer |= 1u << j;
          else if (nxt > sc[j]) status = QF_QSTATUS_UNSORTED;
        }
        if ((p.methods & QF_WRRF) && p.rank && p.rank[g + 1] < p.rank[g])
          status = QF_QSTATUS_RANKORDER;
      }
    }
  }
  if (status) atomicMin(&sh.status, status);
  __syncthreads();
  if (defer) {  // lane 63 only (every sh.first write is behind the barrier)
    int st = 0;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
      if (((defer >> j) & 1u) && sh.first[j * WAVES + wid + 1] > sc[j]) st = QF_QSTATUS_UNSORTED;
    if (st) atomicMin(&sh.status, st);  // read after the barriers that follow
  }
  QF_STOP(12, [&] { uint32_t a = 0u; for (int j = 0; j < ITEMS; ++j) a += dk[j] + (uint32_t)sc[j]; return a; },
          if (_qf_acc == 12345u || threadIdx.x == 0) p.union_count[q] = 0; return -1;);
  // ---- number distinct documents in first-seen order; size their groups ------
  uint32_t repm = 0u;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int e = j * BLOCK + tid;
    uint32_t pc = 0u;
    bool rep = false;
    if (e < N) {
      const uint32_t msk = mask_of(dk[j]);
      rj[j] |= msk << 16;  // the final mask, kept: r | mask << 16 (no second LDS read)
      rep = (uint32_t)(__ffs(msk) - 1) == (rj[j] & 0xFu);
      pc = rep ? (uint32_t)__popc(msk) : 0u;
    }
    repm |= (uint32_t)rep << j;
    const uint64_t b = ballot(rep);
    const uint32_t incl = wave_incl_scan_dpp(pc);
    // the wave-exclusive group prefix, kept for the placement below:
    // rj = r (4 bits) | prefix (<= 16 x 64, 11 bits) << 4 | mask << 16
    rj[j] |= (incl - pc) << 4;
    const uint32_t tot = readlane_u32(incl, 63);
    if (lane == 0) {
      sh.cnt[j * WAVES + wid] = __popcll(b);
      sh.gof[j * WAVES + wid] = (int)tot;
    }
  }
  __syncthreads();
  if (wid == 0) {  // exclusive scans over the (row, wave) chunks, in entry order
    // the block waits on this wave: raised issue priority over the CU's other
    // workgroups (as the QPP kernel's serial chains)
    __builtin_amdgcn_s_setprio(3);
    uint32_t c1 = 0, c2 = 0;
    for (int c0 = 0; c0 < ITEMS * WAVES; c0 += 64) {
      const int i = c0 + lane;
      const uint32_t v1 = i < ITEMS * WAVES ? (uint32_t)sh.cnt[i] : 0u;
      const uint32_t v2 = i < ITEMS * WAVES ? (uint32_t)sh.gof[i] : 0u;
      const uint32_t i1 = wave_incl_scan_dpp(v1), i2 = wave_incl_scan_dpp(v2);
      if (i < ITEMS * WAVES) {
        sh.cnt[i] = (int)(c1 + i1 - v1);
        sh.gof[i] = (int)(c2 + i2 - v2);
      }
      c1 += readlane_u32(i1, 63);
      c2 += readlane_u32(i2, 63);
    }
    if (lane == 0) sh.U = (int)c1;
    __builtin_amdgcn_s_setprio(0);
  }
  __syncthreads();
  QF_STOP(13, [&] { uint32_t a = 0u; for (int j = 0; j < ITEMS; ++j) a += dk[j] + (uint32_t)sc[j]; return a; },
          if (_qf_acc == 12345u || threadIdx.x == 0) p.union_count[q] = 0; return -1;);
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const bool rep = (repm >> j) & 1u;
    const uint64_t b = ballot(rep);
    const uint32_t gpre = (rj[j] >> 4) & 0x7FFu;
    if (rep) {
      const uint32_t u = (uint32_t)sh.cnt[j * WAVES + wid] + mbcnt(b);
      const uint32_t go = (uint32_t)sh.gof[j * WAVES + wid] + gpre;
      // not re-read by the sort kernels: non-temporal (keeps the scores in the MALL)
      __builtin_nontemporal_store(tkey[dk[j]], &p.union_docid[base + u]);
      tkey[dk[j]] = go | (u << 16);  // slot -> group offset | u (the docid is dead)
    }
  }
  __syncthreads();
  // ---- every entry's place in its group (retriever order); a document's
  // first-seen entry opens the group: k == go ---------------------------------
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int e = j * BLOCK + tid;
    if (e < N) {
      const uint32_t gu = tkey[dk[j]];
      const uint32_t r = rj[j] & 0xFu;
      const uint32_t k = (gu & 0xFFFFu) + (uint32_t)__popc((rj[j] >> 16) & ((1u << r) - 1u));
      const uint32_t u = ((repm >> j) & 1u) ? gu >> 16 : 0u;
      dk[j] = k | (u << 16);
    }
  }
  __syncthreads();  // the hash table is dead; its LDS becomes the groups
  QF_STOP(14, [&] { uint32_t a = 0u; for (int j = 0; j < ITEMS; ++j) a += dk[j] + (uint32_t)sc[j]; return a; },
          if (_qf_acc == 12345u || threadIdx.x == 0) p.union_count[q] = 0; return -1;);
  raw_t* gsc = (raw_t*)(smem + L::kGscOff);
  uint32_t* gpr = (uint32_t*)(smem + L::kGprOff);
  uint16_t* ugo = (uint16_t*)(smem + L::kGoOff);
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int e = j * BLOCK + tid;
    if (e < N) {
      const uint32_t k = dk[j] & 0xFFFFu, r = rj[j] & 0xFu;
      gsc[k] = sc[j];
      gpr[k] = (uint32_t)(base + e - sh.off[r]) | (r << 16);
      if ((repm >> j) & 1u) ugo[dk[j] >> 16] = (uint16_t)k;
    }
  }
  __syncthreads();
  QF_STOP(15, [&] { uint32_t a = 0u; for (int j = 0; j < ITEMS; ++j) a += dk[j] + (uint32_t)sc[j]; return a; },
          if (_qf_acc == 12345u || threadIdx.x == 0) p.union_count[q] = 0; return -1;);
  return N;
}

constexpr int kFastSumMethods = QF_COMBSUM | QF_COMBMNZ | QF_RRF | QF_WCOMBSUM | QF_WCOMBMNZ |
                                QF_WRRF;

// 1 / (60 + pos + 1) for every position of a list the LDS join holds: RRF's
// and W-RRF's reciprocal at the reference's k = 60 (config rrf_k) by one cached
// load instead of a reciprocal estimate and two Newton steps inside the
// divergent per-document loop.  Compile-time IEEE divisions (correctly
// rounded, == recip_small bit for bit); 80 KB, its first 8 KB hot in L1.
constexpr int kRecipK = 60, kRecipN = 10240;
struct RecipTable {
  double v[kRecipN];
  constexpr RecipTable() : v() {
    for (int i = 0; i < kRecipN; ++i) v[i] = 1.0 / (double)(kRecipK + i + 1);
  }
};
__device__ constexpr RecipTable kRecip60{};

// Each method slot's range over the query's documents, kept by the join's sums loop
// for the bucket sort (round 5, pair_info below): every thread's running min and
// min of the negated values (= -max), one v_min_f64 each per document and slot.
// Tracked for the compile-time method sets of fast_sums (<= 6 slots).
constexpr int kRangeSlots = 6;
struct SlotRange {
  double mn[kRangeSlots], nmx[kRangeSlots];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int s = 0; s < kRangeSlots; ++s) mn[s] = nmx[s] = INFINITY;
  }
  __device__ __forceinline__ void add(int s, double v) {
    mn[s] = raw_min_f64(mn[s], v);
    nmx[s] = raw_min_neg_f64(nmx[s], v);
  }
};

// The fast path of store_unsorted_sums: MS = the method set when known at compile
// time (0: read it from p.methods; no ranges kept); TAB: rrf_k == 60, reciprocals
// from kRecip60.
template <int MS, bool TAB, class C, int KIND, int EXTRA>
__device__ __forceinline__ void fast_sums(const FuseParams& p, JoinShared<C, KIND, EXTRA>& sh,
                                          int N, const int (&slot)[kNMethods], SlotRange& rg) {
  static_assert(C::kNMax <= kRecipN, "positions beyond the table");
  constexpr int BLOCK = C::kBlock;
  using L = JoinLds<C, KIND>;
  using raw_t = typename L::raw_t;
  const int tid = threadIdx.x;
  const int64_t base = sh.off[0];
  const int U = sh.U;
  const raw_t* gsc = (const raw_t*)(sh.smem + L::kGscOff);
  const uint32_t* gpr = (const uint32_t*)(sh.smem + L::kGprOff);
  const uint16_t* ugo = (const uint16_t*)(sh.smem + L::kGoOff);
  const int methods = MS ? MS : p.methods, rrf_k = p.rrf_k;
  auto doc = [&](int u) {
    const int gs = ugo[u], ge = u + 1 < U ? (int)ugo[u + 1] : N;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a5 = 0.0;
    for (int k = gs; k < ge; ++k) {
      const double s = ScoreIn<KIND>::val(gsc[k]);
      const uint32_t q2 = gpr[k];
      const int r = (int)(q2 >> 16), pos = (int)(q2 & 0xFFFFu);
      const int n = rrf_k + pos + 1;
      const double y = (methods & (QF_RRF | QF_WRRF))
                           ? (TAB ? kRecip60.v[pos] : recip_small(n)) : 0.0;
      const double w = sh.w[r];
      if (methods & (QF_COMBSUM | QF_COMBMNZ)) a0 += s;  // (s - 0.0) / 1.0 == s
      if (methods & QF_RRF) a1 += y;
      if (methods & (QF_WCOMBSUM | QF_WCOMBMNZ)) a2 += w * s;
      if (methods & QF_WRRF) {  // div_small(w, n) with the same reciprocal
        const double qt = w * y;
        a5 += fma(fma(-qt, (double)n, w), y, qt);
      }
    }
    const double cnt = (double)(ge - gs);
    double* out = p.fused + base + u;
    const int64_t st = p.out_stride;
    // each value stored at its slot and, for a compile-time set (slot k = the
    // constant count of requested methods below it), kept in the slot's range
    int k = 0;
    auto put = [&](int t, double x) {
      out[slot[t] * st] = x;
      if (MS != 0) rg.add(k++, x);
    };
    if (methods & QF_COMBSUM) put(0, a0);
    if (methods & QF_COMBMNZ) put(1, a0 * cnt);
    if (methods & QF_RRF) put(2, a1);
    if (methods & QF_WCOMBSUM) put(3, a2);
    if (methods & QF_WCOMBMNZ) put(4, a2 * cnt);
    if (methods & QF_WRRF) put(5, a5);
  };
  // (Measured, not kept: the documents in one list taken first and those in
  // several after them, through a two-class permutation, so that a wave of
  // one-list documents makes one loop step — the stores then scatter over a
  // query's slab and the join took 203 instead of 122 us.)
  for (int u = tid; u < U; u += BLOCK) doc(u);
}

// Every document's fused score for every requested method, from the groups the
// join left in LDS, stored unsorted at fused[slot][base + u] (the sort kernels
// read them back): one thread per document, strided.
// Returns whether `rg` holds every slot's range (a compile-time method set of the
// fast path).
template <class C, int KIND, int EXTRA>
__device__ __forceinline__ bool store_unsorted_sums(const FuseParams& p,
                                                    JoinShared<C, KIND, EXTRA>& sh, int N,
                                                    SlotRange& rg) {
  constexpr int BLOCK = C::kBlock;
  using L = JoinLds<C, KIND>;
  using raw_t = typename L::raw_t;
  const int tid = threadIdx.x;
  const int64_t base = sh.off[0];
  const int U = sh.U;
  const raw_t* gsc = (const raw_t*)(sh.smem + L::kGscOff);
  const uint32_t* gpr = (const uint32_t*)(sh.smem + L::kGprOff);
  const uint16_t* ugo = (const uint16_t*)(sh.smem + L::kGoOff);
  // ---- fused score of every document, every requested method ------------------
  const int methods = p.methods, rrf_k = p.rrf_k;
  int slot[kNMethods];
  for (int t = 0, c = 0; t < kNMethods; ++t) {
    slot[t] = c;
    c += (methods >> t) & 1;
  }
  // The common case without any per-entry range check: micro-unit scores, every
  // list already [0, 1] (x = s), every weight in the division-free range, ranks =
  // positions, k + N + 1 <= 2^24 — CombSUM / CombMNZ / RRF / W-* only.  1 / (k +
  // rank) is computed once per entry for RRF and W-RRF (div_small's reciprocal).
  if (methods == QF_LEARNED) {  // learned fusion alone (C5): its Kahan sums, nothing else
    for (int u = tid; u < U; u += BLOCK) {
      const int gs = ugo[u], ge = u + 1 < U ? (int)ugo[u + 1] : N;
      double a6 = 0.0, c6 = 0.0;
      for (int k = gs; k < ge; ++k) {
        const double s = ScoreIn<KIND>::val(gsc[k]);
        const int r = (int)(gpr[k] >> 16);
        learned_add(p, s, sh.w[r], r, a6, c6);  // src/fusion.py:436-446
      }
      p.fused[base + u] = a6;  // the one method slot
    }
    return false;
  }
  const bool fast = KIND == 1 && sh.slow == 0 && !p.rank && (methods & ~kFastSumMethods) == 0 &&
                    rrf_k >= 0 && rrf_k + N + 1 <= (1 << 24);
  if (fast) {
    // the method set as a compile-time constant for the common sets (C2's six,
    // CombSUM + RRF, W-CombSUM, single methods): a run-time set turns every
    // accumulation into an add plus two selects (34 -> ~24 instructions per entry)
    const bool tab = rrf_k == kRecipK;
    switch (methods) {
      case kFastSumMethods:
        if (tab) fast_sums<kFastSumMethods, true>(p, sh, N, slot, rg);
        else fast_sums<kFastSumMethods, false>(p, sh, N, slot, rg);
        return true;
      case QF_COMBSUM | QF_RRF:
        if (tab) fast_sums<QF_COMBSUM | QF_RRF, true>(p, sh, N, slot, rg);
        else fast_sums<QF_COMBSUM | QF_RRF, false>(p, sh, N, slot, rg);
        return true;
      case QF_WCOMBSUM: fast_sums<QF_WCOMBSUM, false>(p, sh, N, slot, rg); return true;
      case QF_COMBSUM: fast_sums<QF_COMBSUM, false>(p, sh, N, slot, rg); return true;
      case QF_RRF: fast_sums<QF_RRF, false>(p, sh, N, slot, rg); return true;
      case QF_WRRF: fast_sums<QF_WRRF, false>(p, sh, N, slot, rg); return true;
      default: fast_sums<0, false>(p, sh, N, slot, rg); return false;
    }
  }
  for (int u = tid; u < U; u += BLOCK) {
    const int gs = ugo[u], ge = u + 1 < U ? (int)ugo[u + 1] : N;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a5 = 0.0, a6 = 0.0, c6 = 0.0, a7 = 0.0, a8 = 0.0;
    for (int k = gs; k < ge; ++k) {
      const double s = ScoreIn<KIND>::val(gsc[k]);
      const uint32_t q2 = gpr[k];
      const int r = (int)(q2 >> 16), pos = (int)(q2 & 0xFFFFu);
      if (methods & (QF_COMBSUM | QF_COMBMNZ)) {  // ranx min-max normalised score
        const double den = sh.den[r], mn = sh.mn[r];
        // A .norm.res list is already [0, 1] (min 0.000000, max 1.000000), where
        // (s - 0.0) / 1.0 == s bit for bit (-0.0 included): skip the division.
        double x = 0.0;
        if (den > 0.0) {
          const double d = s - mn;
          x = (den == 1.0 && mn == 0.0) ? s
              : (den >= 0x1p-900 && den <= 0x1p900 && d >= 0x1p-900 && d <= 0x1p900)
                  ? div_by_recip(d, den, sh.rden[r])
                  : d / den;
        }
        a0 += x;
      }
      if (methods & QF_RRF) a1 += recip_int(rrf_k + pos + 1);  // ranx rrf: rank = position
      if (methods & (QF_WCOMBSUM | QF_WCOMBMNZ)) a2 += sh.w[r] * s;  // src/fusion.py:273
      if (methods & QF_WRRF) {                                       // src/fusion.py:374
        const int rk = p.rank ? p.rank[sh.off[r] + pos] : pos + 1;
        a5 += div_int(sh.w[r], rrf_k + rk);
      }
      if (methods & (QF_PROBFUSE | QF_WRRF_MUL)) {
        const int rk = p.rank ? p.rank[sh.off[r] + pos] : pos + 1;  // int(row["rank"])
        if (methods & QF_PROBFUSE) {  // ProbFuse.py:30-39,172-179
          // ceil(rank * x / L) in integers (exact: the float quotient of two
          // integers below 2^26 is never rounded onto an integer), clipped to [1, x]
          const int64_t pp = rk > 0 ? rk : 1;
          int64_t k = (pp * p.n_seg + p.seg_len - 1) / p.seg_len;
          k = k < 1 ? 1 : (k > p.n_seg ? p.n_seg : k);
          a7 += div_int(p.seg_prob[r * p.n_seg + (int)k - 1], (int)k);
        }
        if (methods & QF_WRRF_MUL)  // QPPrrf_argmax.py:71: weight * (1.0 / (k + rank))
          a8 += sh.w[r] * recip_int(rrf_k + rk);
      }
      if (methods & QF_LEARNED) learned_add(p, s, sh.w[r], r, a6, c6);  // src/fusion.py:436-446
    }
    const double cnt = (double)(ge - gs);  // CombMNZ: sum x count (src/fusion.py:327)
    double* out = p.fused + base + u;
    const int64_t st = p.out_stride;
    if (methods & QF_COMBSUM) out[slot[0] * st] = a0;
    if (methods & QF_COMBMNZ) out[slot[1] * st] = a0 * cnt;
    if (methods & QF_RRF) out[slot[2] * st] = a1;
    if (methods & QF_WCOMBSUM) out[slot[3] * st] = a2;
    if (methods & QF_WCOMBMNZ) out[slot[4] * st] = a2 * cnt;
    if (methods & QF_WRRF) out[slot[5] * st] = a5;
    if (methods & QF_LEARNED) out[slot[6] * st] = a6;
    if (methods & QF_PROBFUSE) out[slot[7] * st] = a7;
    if (methods & QF_WRRF_MUL) out[slot[8] * st] = a8;
  }
  return false;
}

// ---- the bucket sort's key constants, from the join ----------------------------
// bsort_fast_kernel buckets a (query, method slot) pair's scores by a key whose
// constants depend only on the pair's min and max.  The join holds every score in a
// register once (the sums loop), so it keeps each slot's range (SlotRange) and
// leaves the constants at fused[slot][base + U .. + kPairInfo) — slots [U, N) of a
// query's rows are scratch (include/qppfuse.h) — when N - U >= kPairInfo:
//   [0] min, [1] max (-0.0 folded into +0.0), [2] c: the key's x = v + c when cform,
//   else x = (v - min) + c, [3] top | cform << 31 | scale << 32 (bs_key2), or
//   kPairMark (a range the key cannot take: the fallback pass sorts the pair), or 0:
//   no constants (the sort computes them itself).
// The sort then needs no range phase (round 4: 1.9 x 10^7 VALU and 2.8 x 10^7 SALU
// of the C2 launch, a block reduction and a serial wave-0 section per pair).
constexpr int kPairInfo = 4;
constexpr uint64_t kPairMark = ~0ull;
struct BsKey2 {
  double c;
  uint32_t top, scale;
  int cform, ok;
};
// delta = (max - min) / 2^shift; x = v + (delta - min) when that keeps every x >=
// delta / 2 > 0 (monotone rounding), else (v - min) + delta; bucket = mul_hi(top -
// hi32(x), scale) with top = hi32(x(max)) and scale = floor(MINBASE * 2^32 / span) -
// 1: non-increasing in v (larger scores first), < MINBASE, equal scores together.
template <int MINBASE>
__device__ __forceinline__ BsKey2 bs_key2(double smin, double smax, bool nan, int shift) {
  BsKey2 k{};
  const double rng = smax - smin;
  const double delta = ldexp(rng, -shift);
  if (!(isfinite(rng) && delta > 0.0) || nan) return k;
  const double c = delta - smin;
  k.cform = isfinite(c) && (smin + c) >= 0.5 * delta;
  const double xmin = k.cform ? smin + c : delta;
  const double xmax = k.cform ? smax + c : rng + delta;
  if (!isfinite(xmax)) return k;
  const uint32_t b0 = (uint32_t)((uint64_t)__double_as_longlong(xmin) >> 32);
  k.top = (uint32_t)((uint64_t)__double_as_longlong(xmax) >> 32);
  const uint32_t span = k.top - b0 + 1u;
  k.scale = span <= (uint32_t)MINBASE
                ? 0xFFFFFFFFu
                : (uint32_t)((double)MINBASE * 4294967296.0 / (double)span) - 1u;
  k.c = k.cform ? c : delta;
  k.ok = 1;
  return k;
}
__device__ __forceinline__ uint64_t bs_key2_word(const BsKey2& k) {
  return k.ok ? ((uint64_t)k.scale << 32) | ((uint64_t)k.cform << 31) | k.top : kPairMark;
}
// two configurations (bsort_fast_kernel): unions up to kJsUMax with 2^12 buckets, and
// (kJsUMax, kFastUMaxL] — SURVEY §8(d)'s C2 unions, ~4,030 — with 2^13
constexpr int kFastBits = 12, kFastNB = 1 << kFastBits, kFastMinBase = kFastNB - kFastNB / 16;
constexpr int kFastBitsL = 13, kFastNBL = 1 << kFastBitsL,
              kFastMinBaseL = kFastNBL - kFastNBL / 16;
constexpr int kFastUMaxL = 5120;
constexpr int kFastDeltaShift = 8;   // delta = range / 2^8 (tools/bsort_sim.py, round 3)
constexpr int kFastRetryShift = 20;  // the recount after a bucket overflow

// Quad min of a double (DPP quad_perm; result in every lane of the quad).
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int64_t b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double(((int64_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ double quad_min_f64(double x) {
  x = raw_min_f64(x, dpp_f64<0xB1>(x));  // quad_perm [1,0,3,2]
  x = raw_min_f64(x, dpp_f64<0x4E>(x));  // quad_perm [2,3,0,1]
  return x;
}

// min(a, b) of the value pair the half-exchange v_permlane32_swap (SIXTEEN: the
// row exchange v_permlane16_swap) leaves in this lane: lanes of the lower half
// (row) keep value a, min'd with the partner lane's a; the upper half keeps b.
template <bool SIXTEEN>
__device__ __forceinline__ double swap_min_f64(double a, double b) {
  const uint64_t ua = (uint64_t)__double_as_longlong(a), ub = (uint64_t)__double_as_longlong(b);
  const auto lo = SIXTEEN ? __builtin_amdgcn_permlane16_swap((uint32_t)ua, (uint32_t)ub, false, false)
                          : __builtin_amdgcn_permlane32_swap((uint32_t)ua, (uint32_t)ub, false, false);
  const auto hi = SIXTEEN
                      ? __builtin_amdgcn_permlane16_swap((uint32_t)(ua >> 32), (uint32_t)(ub >> 32),
                                                         false, false)
                      : __builtin_amdgcn_permlane32_swap((uint32_t)(ua >> 32), (uint32_t)(ub >> 32),
                                                         false, false);
  const double x = __longlong_as_double((int64_t)(((uint64_t)hi[0] << 32) | lo[0]));
  const double y = __longlong_as_double((int64_t)(((uint64_t)hi[1] << 32) | lo[1]));
  return raw_min_f64(x, y);
}

// Every slot's range reduced over the block and its key constants stored (see
// above).  All threads call it after the sums; `ranged`: rg holds the ranges.
// The 12 running values (6 minima, 6 negated maxima) are reduced in registers:
// two half-exchanges leave each lane 3 values, min'd over 4 lanes (v_permlane32 /
// 16_swap: lanes 0-31 keep values 0-5, lanes 32-63 values 6-11, then even 16-lane
// rows the first 3 of those, odd rows the last 3), a DPP butterfly reduces them over
// each row (row r then holds values 3r .. 3r + 2), one lane per row stores them, and
// wave 0 reduces the waves' results — no LDS transposition (round 5's first form,
// whose transposed reads hit one bank per lane quad: join +48 us).
template <class C, int KIND, int EXTRA>
__device__ __forceinline__ void pair_info(const FuseParams& p, JoinShared<C, KIND, EXTRA>& sh,
                                          int N, bool ranged, const SlotRange& rg) {
  constexpr int WAVES = C::kWaves, NV = 2 * kRangeSlots;
  static_assert(NV == 12, "three values per 16-lane row after the two exchanges");
  const int U = sh.U;
  if (sh.status || N - U < kPairInfo) return;  // uniform
  const int M = __popc(p.methods);
  const int64_t at = sh.off[0] + U;
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (!ranged || M > kRangeSlots) {  // uniform: "no constants" (w3 = 0)
    if (tid < M) ((uint64_t*)p.fused)[tid * p.out_stride + at + 3] = 0ull;
    return;
  }
  double y[6], z[3];
#pragma unroll
  for (int k = 0; k < 6; ++k) y[k] = swap_min_f64<false>(rg.mn[k], rg.nmx[k]);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    z[k] = swap_min_f64<true>(y[k], y[k + 3]);
    z[k] = raw_min_f64(z[k], dpp_f64<0xB1>(z[k]));   // quad_perm [1,0,3,2]
    z[k] = raw_min_f64(z[k], dpp_f64<0x4E>(z[k]));   // quad_perm [2,3,0,1]
    z[k] = raw_min_f64(z[k], dpp_f64<0x141>(z[k]));  // row_half_mirror
    z[k] = raw_min_f64(z[k], dpp_f64<0x140>(z[k]));  // row_mirror
  }
  if ((lane & 15) == 0) {
#pragma unroll
    for (int k = 0; k < 3; ++k) sh.wres[3 * (lane >> 4) + k][wid] = z[k];
  }
  __syncthreads();
  if (wid == 0) {
    // lanes 4v .. 4v + 3: value v over the waves, then a quad min
    double x = INFINITY;
    if (lane < 4 * NV)
      for (int k = lane & 3; k < WAVES; k += 4) x = raw_min_f64(x, sh.wres[lane >> 2][k]);
    x = quad_min_f64(x);
    // lane 4s: min of slot s; lane 4 (kRangeSlots + s): -max of slot s
    const int64_t nb = __double_as_longlong(x);
    const int src = (lane + 4 * kRangeSlots) << 2;
    const int lo = __builtin_amdgcn_ds_bpermute(src, (int)nb);
    const int hi = __builtin_amdgcn_ds_bpermute(src, (int)(nb >> 32));
    const double nmax = __longlong_as_double(((int64_t)hi << 32) | (uint32_t)lo);
    if ((lane & 3) == 0 && (lane >> 2) < M) {
      const int s = lane >> 2;
      const double smin = x + 0.0, smax = -nmax + 0.0;  // -0.0 folded into +0.0
      const BsKey2 k = U <= 3072 ? bs_key2<kFastMinBase>(smin, smax, false, kFastDeltaShift)
                                 : bs_key2<kFastMinBaseL>(smin, smax, false, kFastDeltaShift);
      double* o = p.fused + s * p.out_stride + at;
      o[0] = smin;
      o[1] = smax;
      o[2] = k.c;
      ((uint64_t*)o)[3] = bs_key2_word(k);
    }
  }
}

// f64 scores need 72 KB of LDS (2 per CU), so only micro-unit scores aim higher
template <class C, int KIND>
__global__ __launch_bounds__(C::kBlock, KIND == 1 ? C::kMinWaves : (C::kMinWaves < 4 ? C::kMinWaves : 4))
void join_kernel(FuseParams p) {
  __shared__ JoinShared<C, KIND> sh;
  const int64_t q = block_id();
  if (q >= p.n_queries) return;
  const int N = join_groups<C, KIND>(p, sh, q);
  if (N < 0) return;
  SlotRange rg;
  rg.init();
  const bool ranged = store_unsorted_sums<C, KIND>(p, sh, N, rg);
  if (threadIdx.x == 0) p.union_count[q] = sh.status ? sh.status : sh.U;
  // (development stop 16: the sums without the key constants — w3 = 0, the sort
  // computes them itself)
  QF_STOP(16, [&] { return 0u; },
          pair_info<C, KIND>(p, sh, N, false, rg); return;);
  pair_info<C, KIND>(p, sh, N, ranged, rg);
}

// ============================================================================
// fuse_kernel
// ============================================================================
// The bucket sorts' limits (join_sort_kernel / bucket_sort_kernel below): unions
// up to kJsUMax; a (query, method) they leave unsorted has perm[0] = kJsUnsorted.
constexpr int kJsUMax = 3072;
constexpr uint16_t kJsUnsorted = 0xFFFF;

template <int BLOCK, int ITEMS, int MINW>
struct SortCfg {
  static constexpr int kBlock = BLOCK, kItems = ITEMS, kWaves = BLOCK / 64, kMinWaves = MINW;
  static constexpr int kUMax = BLOCK * ITEMS;
  static constexpr int kItemOff = 0;                // u32 [UMAX]
  static constexpr int kHistOff = 4 * kUMax;         // u16 [W][kBuckets]
  static constexpr int kSmem = kHistOff + 2 * kBuckets * kWaves;
  static_assert(kUMax <= (int)kUMask + 1, "u is kUBits bits of the item");
  static_assert(kSmem <= 160 * 1024, "LDS budget");
};

template <class C>
struct SortShared {
  __attribute__((aligned(16))) unsigned char smem[C::kSmem];
  int flag[2];
  uint32_t wtot[16];
  unsigned long long kmin, kmax;
  unsigned int dmin, dmax;
};

// Sort one (query, method slot): fused[ms][base .. base+U) in place + perm.
// Ties keep first-seen order, or (by_docid: learned fusion, whose groupby
// output is in docno order, src/fusion.py:443-446) docid order: LSD passes over
// the docids first, then the score passes, all stable.
template <class C>
__device__ __forceinline__ void sort_one(const FuseParams& p, SortShared<C>& sh, int ms, int U,
                                         int64_t base, bool by_docid) {
  constexpr int ITEMS = C::kItems, WAVES = C::kWaves;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) {
    sh.kmin = ~0ull;
    sh.kmax = 0ull;
    sh.dmin = ~0u;
    sh.dmax = 0u;
  }
  __syncthreads();
  double* io = p.fused + (int64_t)ms * p.out_stride + base;  // unsorted fused[ms][u]
  const uint32_t* udoc = p.union_docid + base;
  const int rows = (U + 64 * WAVES - 1) / (64 * WAVES);
  // ---- the join kernel's unsorted scores -> LDS, their key range -----------------
  uint64_t fk[ITEMS];
  double fv[ITEMS];  // the scores themselves (the linearised window key needs them)
  uint32_t ud[ITEMS];  // learned fusion: the docids (their range for the docid passes)
  uint64_t kmn = ~0ull, kmx = 0ull;
  uint32_t dmn = ~0u, dmx = 0u;
  // every row's load in flight before the first use (one HBM latency, not one per row)
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int i = (wid * rows + j) * 64 + lane;
    fv[j] = (j < rows && i < U) ? io[i] : 0.0;
    ud[j] = (by_docid && j < rows && i < U) ? udoc[i] : 0u;
  }
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int i = (wid * rows + j) * 64 + lane;
    fk[j] = 0;
    if (j < rows && i < U) {
      fk[j] = ~f64_asc_key(fv[j]);  // ascending sort on ~key == descending score
      kmn = min(kmn, fk[j]);
      kmx = max(kmx, fk[j]);
      if (by_docid) {
        dmn = min(dmn, ud[j]);
        dmx = max(dmx, ud[j]);
      }
    }
  }
  block_min_max(kmn, kmx, &sh.kmin, &sh.kmax, lane);
  if (by_docid) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
      dmn = min(dmn, (uint32_t)__shfl_xor((int)dmn, d, 64));
      dmx = max(dmx, (uint32_t)__shfl_xor((int)dmx, d, 64));
    }
    if (lane == 0) {
      atomicMin(&sh.dmin, dmn);
      atomicMax(&sh.dmax, dmx);
    }
  }
  __syncthreads();
  const uint64_t kmin = sh.kmin, kmax = sh.kmax;
  SortCtx<ITEMS, WAVES> sx{(uint32_t*)(sh.smem + C::kHistOff),
                           (uint32_t*)(sh.smem + C::kItemOff), io, sh.wtot, sh.flag, kmin, U,
                           rows, lane, wid, tid};
  const int hb_full = kmax > kmin ? 64 - __clzll((long long)(kmax - kmin)) : 0;
  // Window key.  The raw key's top bits are mostly exponent, so a short window
  // of it collides a lot; for a finite score range the window is cut from
  // wkey(v) = ~orderable((v - smin) + rng * 2^-6) instead: non-decreasing in
  // the full key (each rounding is monotone), so different windows are in
  // full-key order and only equal windows need the fix-up.  Its extremes are
  // wkey(smax) and wkey(smin) by the same monotonicity.
  const double smax = f64_from_asc_key(~kmin), smin = f64_from_asc_key(~kmax);
  const double rng = smax - smin;
  const bool lin = hb_full > 0 && isfinite(rng);
  const double delta = rng * 0x1p-6;
  auto wkey = [&](uint64_t key) -> uint64_t {
    return lin ? ~f64_asc_key((f64_from_asc_key(~key) - smin) + delta) : key;
  };
  const uint64_t wmin = lin ? ~f64_asc_key((smax - smin) + delta) : kmin;
  const uint64_t wmax = lin ? ~f64_asc_key((smin - smin) + delta) : kmax;
  const int hb = wmax > wmin ? 64 - __clzll((long long)(wmax - wmin)) : 0;
  const int lo = hb > kWindow ? hb - kWindow : 0;
  const bool exact = !lin && lo == 0;  // the window holds the whole key
  uint32_t item[ITEMS];
  if (by_docid && sh.dmax > sh.dmin) {
    // ---- learned fusion: first into docid order ------------------------------------
    const uint32_t dmin = sh.dmin;
    const int db = 32 - __clz((int)(sh.dmax - dmin));
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) item[j] = (uint32_t)((wid * rows + j) * 64 + lane);
#pragma unroll 1
    for (int s0 = 0; s0 < db; s0 += kDigit) {
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        const int i = (wid * rows + j) * 64 + lane;
        if (j < rows && i < U) {
          const uint32_t u = item[j] & kUMask;
          item[j] = ((((udoc[u] - dmin) >> s0) & (uint32_t)(kBuckets - 1)) << kUBits) | u;
        }
      }
      count_scatter(sx, item, 0, true);
    }
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {  // registers now hold docid order: re-key
      const int i = (wid * rows + j) * 64 + lane;
      if (j < rows && i < U) {
        const uint32_t u = item[j] & kUMask;
        item[j] = ((uint32_t)((wkey(~f64_asc_key(io[u])) - wmin) >> lo) << kUBits) | u;
      }
    }
  } else {
    // ---- items: window key | u --------------------------------------------------
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const int i = (wid * rows + j) * 64 + lane;
      // wkey(fk[j]) straight from the score (-0.0 and +0.0 give the same (v - smin) + delta)
      const uint64_t wk = lin ? ~f64_asc_key((fv[j] - smin) + delta) : fk[j];
      item[j] = ((uint32_t)((wk - wmin) >> lo) << kUBits) | (uint32_t)i;
    }
  }
  if (hb_full > 0) sort_desc(sx, item, hb - lo, exact, hb_full);  // else all keys equal
  write_out(sx, item, p, (int64_t)ms * p.out_stride + base);
}
// Method bit of output slot ms.
__device__ __forceinline__ int slot_method(int methods, int ms) {
  for (int t = 0, c = 0; t < kNMethods; ++t)
    if ((methods >> t) & 1) {
      if (c == ms) return t;
      ++c;
    }
  return 0;
}

// One workgroup per (query, method slot), the queries with U in [umin, UMAX].
template <class C>
__global__ __launch_bounds__(C::kBlock, C::kMinWaves) void fuse_kernel(FuseParams p, int umin) {
  __shared__ SortShared<C> sh;
  // block -> (query, method slot): slot-major groups of 8 queries, so that the
  // blocks resident together on an XCD (blockIdx % 8) read adjacent queries.
  const int M = __popc(p.methods);
  const int64_t bid = block_id();
  const int64_t grp8 = bid >> 3;
  const int64_t q = (grp8 / M) * 8 + (bid & 7);
  const int ms = (int)(grp8 % M);
  if (q >= p.n_queries) return;
  const int U = p.union_count[q];
  const int64_t base = p.list_off[q * p.R];  // both loads in flight together
  if (U < 0 || U > C::kUMax || U < umin) return;  // error / other pass
  sort_one<C>(p, sh, ms, U, base, slot_method(p.methods, ms) == 6);
}

// The same for the few large queries (U in [umin, UMAX]): a grid of one
// workgroup per CU, each listing the (query, method) pairs of its stride
// that qualify (one parallel load of their counts) and sorting them in turn —
// so a batch without large queries costs a few microseconds, not one
// dispatched workgroup per pair.  FB: the same pass also takes the pairs the
// bucket sort left unsorted (perm[0] marked, U <= kJsUMax) — what
// a separate fallback kernel did, without its launch and scan (~5 us).
template <class C, bool FB = false>
__global__ __launch_bounds__(C::kBlock, C::kMinWaves) void fuse_large_kernel(FuseParams p,
                                                                            int umin) {
  __shared__ SortShared<C> sh;
  __shared__ int s_list[C::kBlock];
  __shared__ int s_n;
  const int tid = threadIdx.x;
  const int M = __popc(p.methods);
  const int64_t pairs = p.n_queries * M;
  const int64_t span = (int64_t)gridDim.x * C::kBlock;
  for (int64_t c0 = 0; c0 < pairs; c0 += span) {
    if (tid == 0) s_n = 0;
    __syncthreads();
    const int64_t idx = c0 + (int64_t)tid * gridDim.x + blockIdx.x;
    if (idx < pairs) {
      const int64_t q = idx / M;
      const int U = p.union_count[q];
      bool take = U >= umin && U <= C::kUMax;
      // the fallback pass: a pair within a bucket sort's reach is taken when it marked
      // it (learned fusion's docid-tie sort reaches p.learned_reach, the others kFastUMaxL)
      const int reach = slot_method(p.methods, (int)(idx % M)) == 6
                            ? (p.learned_reach ? p.learned_reach : kJsUMax)
                            : (p.fast_reach ? p.fast_reach : kJsUMax);
      if (FB && U > 1 && U <= reach)
        take = perm_get(p, (idx % M) * p.out_stride + p.list_off[q * p.R]) == kJsUnsorted;
      if (take) s_list[atomicAdd(&s_n, 1)] = (int)(idx - c0);
    }
    __syncthreads();
    const int n = s_n;
    for (int t = 0; t < n; ++t) {
      const int64_t id = c0 + s_list[t];
      const int64_t q = id / M;
      const int ms = (int)(id % M);
      sort_one<C>(p, sh, ms, p.union_count[q], p.list_off[q * p.R],
                  slot_method(p.methods, ms) == 6);
      __syncthreads();
    }
  }
}


// ============================================================================
// The bucket sort of the default path (bsort_kernel below; join_sort_xl_kernel's
// workspace bucket sort is the same algorithm over a global workspace).
// Per (query, method) slot, over the join's unsorted fused[slot][0..U):
//   1. count: one returning LDS atomic per item on its bucket, a monotone key of
//      the score (order inside a bucket is arbitrary; the return value is the
//      item's arrival index);
//   2. exclusive scan of the bucket counters;
//   3. scatter the score (and what the rank needs) to start[bucket] + arrival;
//   4. the final position of an item is its bucket's start + the number of items
//      of its bucket that precede it in (score descending, u ascending) order —
//      the stable sort's order, counted exactly with f64 compares.
// Its cost per item is the size of its bucket (C2 with QPP or random weights:
// 2-2.5 on average; tools/bucket_stats.py).  A bucket above kJsBucketMax is
// counted once more with a finer key (QF_BS_RETRY_SHIFT); a bucket still above
// it or a non-finite / NaN score range leaves the (query, method) to the LSD
// window sort of fuse_large_kernel's fallback pass (the same order).
// (Rounds 1-2 also kept a one-kernel join + sort and a float-bit-key bucket sort
// for A/B; both measured slower and were removed in round 3.)
// ============================================================================
constexpr int kJsBucketMax = 128;
#ifndef QF_BS_RETRY_SHIFT  // the recount's finer delta (a bucket overflowed)
#define QF_BS_RETRY_SHIFT 20
#endif


// ============================================================================
// bsort_kernel — the default path's sort: the bucket sort above, one workgroup
// (512 threads) per (query, method slot) with U <= kJsUMax, at a low VALU count
// (the kernel is VALU-issue-bound):
//  * the key is one f64 add and a multiply-high: x = v + c (c = delta - smin,
//    when smin + c >= delta / 2; else (v - smin) + delta), the high word of x's
//    bits (x > 0: its bits ascend with x) scaled over the MINBASE buckets — every
//    step monotone, so the bucket is non-increasing in v; the minimum score
//    (shared by hundreds of documents when a run has weight 0) takes MINSUB
//    sub-buckets split by u;
//  * u32 bucket counters overlaid on the scores' LDS, which is free until the
//    scatter;
//  * the scatter keeps each item's (u, bucket size, arrival index) and stores
//    them as one u32 word by position, so the rank phase reads lo / hi and the
//    tie key with one read.
// Same order (score descending, ties in first-seen u order); a pair it cannot
// order gets perm[0] = kJsUnsorted for the fallback pass.
// LDS: the scores by position (24 KB; before the scatter the range partials and
// the counters), then 14 KB for the bucket starts and, from the scatter on, the
// words by position.  38.2 KB: 4 workgroups per CU.
// ============================================================================

// a == s ? if_eq : if_ne as one compare and one v_cndmask (the compiler turns
// the plain ternary into a branch around the f64 key arithmetic, ~6 more
// instructions per item; s_nop 1: the VCC-write -> lane-select wait states).
__device__ __forceinline__ uint32_t sel_if_eq_f64(double a, double s, uint32_t if_eq,
                                                  uint32_t if_ne) {
  uint32_t r;
  asm("v_cmp_eq_f64_e32 vcc, %1, %2\n\ts_nop 1\n\tv_cndmask_b32_e32 %0, %4, %3, vcc"
      : "=v"(r)
      : "s"(s), "v"(a), "v"(if_eq), "v"(if_ne)
      : "vcc");
  return r;
}

// before + [member j precedes item i]: (kj > ki) or (kj == ki and tj < ti), for
// ascending integer keys k (larger score first) and tie words t (smaller first) —
// the borrow out of the 96-bit difference (ki, ~ti) - (kj, ~tj), added with carry:
// four full-rate integer VALU ops and no scalar mask logic (the f64 compare form
// needed two f64 compares, a u32 compare and three SALU combines per member).
// The low word's ~ti - ~tj equals tj - ti (mod 2^32) with the same borrow.
__device__ __forceinline__ uint32_t add_if_precedes(uint32_t before, uint64_t ki, uint32_t ti,
                                                    uint64_t kj, uint32_t tj) {
  uint32_t r, d;
  asm("v_sub_co_u32_e32 %1, vcc, %3, %4\n\t"
      "v_subb_co_u32_e32 %1, vcc, %5, %6, vcc\n\t"
      "v_subb_co_u32_e32 %1, vcc, %7, %8, vcc\n\t"
      "v_addc_co_u32_e32 %0, vcc, 0, %2, vcc"
      : "=v"(r), "=&v"(d)
      : "v"(before), "v"(tj), "v"(ti), "v"((uint32_t)ki), "v"((uint32_t)kj),
        "v"((uint32_t)(ki >> 32)), "v"((uint32_t)(kj >> 32))
      : "vcc");
  return r;
}

// The ascending integer key of a finite or infinite score, -0.0 folded into +0.0
// (v + 0.0), so equal keys are exactly equal scores (NaN pairs take the fallback).
__device__ __forceinline__ uint64_t bs_rank_key(double v) {
  const uint64_t b = (uint64_t)__double_as_longlong(v + 0.0);
  const uint64_t s = (uint64_t)((int64_t)b >> 63);
  return b ^ (s | 0x8000000000000000ull);
}

// bsort_kernel's bucket-key constants for delta = range / 2^shift (every value
// uniform over the workgroup): x = v + c (cform) or (v - smin) + delta, bucket key
// (hi32(x) - b0) * scale >> 32.  ok = 0: a range the key cannot take.
__device__ __forceinline__ double rfl_f64(double v) {  // a wave-uniform double in SGPRs
  const int64_t b = __double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32));
  return __longlong_as_double((int64_t)(((uint64_t)hi << 32) | lo));
}
struct BsKey {
  double c, delta;
  uint32_t b0, scale;
  int cform, ok;
};
template <int MINBASE, bool BYDOC>
__device__ __forceinline__ BsKey bs_key_params(double smin, double smax, bool nan, int shift) {
  BsKey k{};
  const double rng = smax - smin;
  // BYDOC with every score equal: every item is a minimum (by docid); any
  // positive delta gives the (unused) key a valid range
  k.delta = (BYDOC && rng == 0.0) ? 1.0 : ldexp(rng, -shift);
  if (!(isfinite(rng) && k.delta > 0.0) || nan) return k;
  k.c = k.delta - smin;
  // x = v + c when that keeps x >= delta / 2 > 0 for every v >= smin (monotone
  // rounding: x(v) >= x(smin)); else the exact-difference form
  k.cform = isfinite(k.c) && (smin + k.c) >= 0.5 * k.delta;
  const double xmin = k.cform ? smin + k.c : k.delta;
  const double xmax = k.cform ? smax + k.c : rng + k.delta;
  if (!isfinite(xmax)) return k;
  k.b0 = (uint32_t)((uint64_t)__double_as_longlong(xmin) >> 32);
  const uint32_t top = (uint32_t)((uint64_t)__double_as_longlong(xmax) >> 32);
  // key = (hx - b0) * scale >> 32 spreads the span over all MINBASE buckets (a
  // power-of-two shift would use 1/2-1 of them): scale = floor(MINBASE * 2^32 /
  // span), one below for rounding, so the largest key is MINBASE - 1 at most
  const uint32_t span = top - k.b0 + 1u;
  k.scale = span <= (uint32_t)MINBASE
                ? 0xFFFFFFFFu
                : (uint32_t)((double)MINBASE * 4294967296.0 / (double)span) - 1u;
  k.ok = 1;
  return k;
}

// delta = range / 2^8: with the multiply-scaled key, 8 binades above the minimum
// balance the buckets best on the C2 fusions (tools/bsort_sim.py: the rank loop's
// largest bucket per 64 positions 4.3 -> 3.5 against the shifted 12-binade key)
#ifndef QF_BSORT_DELTA_SHIFT
#define QF_BSORT_DELTA_SHIFT 8
#endif
// BYDOC: learned fusion's slot, whose ties go in docid (= docno) order — the
// reference's groupby returns each query's list in docno order before
// write_runfile sorts it stably (src/fusion.py:441-446, 475-488): the docids are
// loaded with the scores, the minimum's sub-buckets split by docid, the rank
// compares docids (a u32 by position: 12 KB more LDS, 3 workgroups per CU).
// Without BYDOC the learned slot is skipped (its own launch takes it).
// The bucket sort's small shared state (block reductions, flags, key constants).
template <int WAVES>
struct BsShared {
  uint32_t wtot[WAVES], big[WAVES];
  double mn, mx;
  int wnan[WAVES], nan;
  uint32_t dmn, dmx;
  BsKey key;  // wave 0's key constants for the first count
};

// LDS bytes of bsort_core's area (region A + region BC; BYDOC's docids after it):
// region BC holds the words by position (u32 [UMAX]) and, before them, BYDOC's docid
// partials (u32 [2 * BLOCK]) and then the bucket starts (u16 [NB + 8], at kStart).
template <int BITS, bool BYDOC, int UMAX = kJsUMax, int BLOCK = 512>
struct BsLds {
  static constexpr int kNB = 1 << BITS;
  static constexpr int kStart = UMAX == kJsUMax ? 6144 : 8 * BLOCK;
  static constexpr int kBcBytes = (4 * UMAX > kStart + 2 * (kNB + 8)) ? 4 * UMAX
                                                                      : kStart + 2 * (kNB + 8);
  static constexpr int kSd = 8 * UMAX + kBcBytes;  // BYDOC: docid by position
  static constexpr int kBytes = kSd + (BYDOC ? 4 * UMAX : 0);
};

// The bucket sort of one (query, method slot) pair whose U scores are in
// registers: item j of this lane is u = ub0 + j * ustep + lane (ub0, ustep
// 64-aligned and wave-uniform; every u in [0, rows * BLOCK) held by exactly one
// lane), v[j] its score, d[j] its docid (BYDOC).  lds: BsLds<BITS, BYDOC>::kBytes
// of LDS no one else uses until the call returns.  Writes perm[po + i] (or marks
// perm[po] for the fallback pass).  Every thread of the block calls it.
// Returns whether it marked the pair (block-uniform).
template <int BLOCK, int BITS, bool BYDOC, int UMAX = kJsUMax>
__device__ __forceinline__ bool bsort_core(const FuseParams& p, unsigned char* lds,
                                           BsShared<BLOCK / 64>& sm,
                                           double (&v)[(UMAX + BLOCK - 1) / BLOCK],
                                           uint32_t (&d)[BYDOC ? (UMAX + BLOCK - 1) / BLOCK : 1],
                                           int U, int ub0, int ustep, int64_t po) {
  constexpr int WAVES = BLOCK / 64, ROWS = (UMAX + BLOCK - 1) / BLOCK, NB = 1 << BITS;
  constexpr int MINSUB = NB / 16, MINBASE = NB - MINSUB;
  static_assert(2 * BLOCK * 8 + 4 * NB <= 8 * UMAX, "partials + counters overlay the scores");
  // One LDS array: region A = the scores by position (f64 [kJsUMax]; until the
  // scatter: the range partials [0, 8 KB) and the u32 counters [8 KB, 24 KB));
  // region BC after it = the u | size | arrival words by position (u32 [kJsUMax],
  // from the scatter on), before that the bucket starts (u16, at BC + 6 KB), the
  // spare counter cnt[NB] (BC[0]) and BYDOC's docid partials (BC[0, 4 KB)).
  using LD = BsLds<BITS, BYDOC, UMAX, BLOCK>;
  static_assert(LD::kBcBytes >= 4 * UMAX && LD::kStart >= 8 * BLOCK, "region BC layout");
  double* sval = (double*)lds;                                   // region A
  uint64_t* skey = (uint64_t*)lds;  // region A from the scatter on: bs_rank_key by position
  uint32_t* sw = (uint32_t*)(lds + 8 * UMAX);                    // region BC: u << 16 | size << 8 | at
  uint16_t* bk = (uint16_t*)(lds + 8 * UMAX + LD::kStart);       // bucket starts [NB + 8]
  uint32_t* cnt = (uint32_t*)(sval + 2 * BLOCK);                 // [NB + 1] u32
  uint32_t* sd = (uint32_t*)(lds + LD::kSd);                     // docid by position (BYDOC)
  const int tid = threadIdx.x, lane = tid & 63,
            wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rows = (U + BLOCK - 1) / BLOCK;
  const int pbase = wid * rows * 64;  // this wave's positions: [pbase, pbase + rows * 64)
  {  // zero the counters (region A beyond the partials)
    uint4* c4 = (uint4*)cnt;
#pragma unroll
    for (int i = tid; i < NB / 4; i += BLOCK) c4[i] = make_uint4(0u, 0u, 0u, 0u);
  }
  {  // score range (NaN flagged): every thread's partials, reduced by wave 0
    double vmn = INFINITY, vmx = -INFINITY;
    bool nan = false;
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      const int u = ub0 + j * ustep + lane;
      if (j < rows && u < U) {
        vmn = raw_min_f64(vmn, v[j]);
        vmx = raw_max_f64(vmx, v[j]);
        nan |= v[j] != v[j];
      }
    }
    sval[tid] = vmn;
    sval[BLOCK + tid] = vmx;
    if (BYDOC) {  // docid range: partials in region B (free until the scatter)
      uint32_t dmn = ~0u, dmx = 0u;
#pragma unroll
      for (int j = 0; j < ROWS; ++j) {
        const int u = ub0 + j * ustep + lane;
        if (j < rows && u < U) {
          dmn = min(dmn, d[j]);
          dmx = max(dmx, d[j]);
        }
      }
      sw[tid] = dmn;
      sw[BLOCK + tid] = dmx;
    }
    const bool anynan = ballot(nan) != 0ull;
    if (lane == 0) sm.wnan[wid] = anynan ? 1 : 0;
  }
  __syncthreads();
  if (wid == 0) {
    __builtin_amdgcn_s_setprio(3);  // the block waits on this wave
    double mn = sval[lane], mx = sval[BLOCK + lane];
#pragma unroll
    for (int i = 1; i < WAVES; ++i) {
      mn = raw_min_f64(mn, sval[i * 64 + lane]);
      mx = raw_max_f64(mx, sval[BLOCK + i * 64 + lane]);
    }
    mn = wave_min_f64_dpp(mn);
    mx = wave_max_f64_dpp(mx);
    uint32_t dmn = 0u, dmx = 0u;
    if (BYDOC) {
      const uint32_t* sp = sw;
      dmn = sp[lane];
      dmx = sp[BLOCK + lane];
#pragma unroll
      for (int i = 1; i < WAVES; ++i) {
        dmn = min(dmn, sp[i * 64 + lane]);
        dmx = max(dmx, sp[BLOCK + i * 64 + lane]);
      }
      dmn = (uint32_t)wave_min_u64_dpp(dmn);
      dmx = (uint32_t)wave_max_u64_dpp(dmx);
    }
    int anyn = 0;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) anyn |= sm.wnan[w];
    if (lane == 63) {
      // the folded extremes (-0.0 == +0.0) and the first count's key constants,
      // once here instead of in every wave after the barrier
      const double fmx = f64_from_asc_key(f64_asc_key(mx)), fmn = f64_from_asc_key(f64_asc_key(mn));
      sm.mn = fmn;
      sm.mx = fmx;
      sm.nan = anyn;
      sm.dmn = dmn;
      sm.dmx = dmx;
      sm.key = bs_key_params<MINBASE, BYDOC>(fmn, fmx, anyn != 0, QF_BSORT_DELTA_SHIFT);
    }
    __builtin_amdgcn_s_setprio(0);
  }
  __syncthreads();
  const bool nan = sm.nan != 0;
  if (!BYDOC && sm.mn == sm.mx && !nan) {  // every score equal: first-seen order
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      const int u = ub0 + j * ustep + lane;
      if (j < rows && u < U) perm_put(p, po + u, (uint32_t)u);
    }
    return false;
  }
  const double smax = sm.mx, smin = sm.mn;
  int ush = 0;  // U - 1 >> ush < MINSUB
  while (((uint32_t)(U - 1) >> ush) >= (uint32_t)MINSUB) ++ush;
  const uint32_t dmin = BYDOC ? sm.dmn : 0u;
  int dsh = 0;  // BYDOC: (dmax - dmin) >> dsh < MINSUB
  if (BYDOC)
    while (((sm.dmx - dmin) >> dsh) >= (uint32_t)MINSUB) ++dsh;
  // the minimum's sub-bucket of row j: MINBASE + (ub0 + ustep j + lane) >> ush, with
  // 64-aligned row bases and ush <= 6 (U <= kJsUMax): a per-lane part + a row part
  static_assert(((UMAX - 1) >> 6) < MINSUB, "ush <= 6");
  const uint32_t lane_sub = (uint32_t)lane >> ush;
  uint32_t ws[ROWS];  // bucket | arrival index << 16
  // count with delta = range / 2^shift: -1 = a range the key cannot take (the
  // pair is marked), else whether some bucket exceeds kJsBucketMax
  // one row pass of the count: CF = the v + c form.  Every row's atomic is issued
  // before any result is used (one wait); a lane past U adds to the spare counter
  // cnt[NB] (in region B, free until the scatter), so no branch surrounds them
  auto count_rows = [&](auto cf, double c, double delta, uint32_t b0, uint32_t scale) -> bool {
    constexpr bool CF = decltype(cf)::value;
    uint32_t old[ROWS];
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      if (j < rows) {  // uniform
        const int u = ub0 + j * ustep + lane;
        const double x = CF ? v[j] + c : (v[j] - smin) + delta;
        const uint32_t hx = (uint32_t)((uint64_t)__double_as_longlong(x) >> 32);
        const uint32_t minb = BYDOC ? (uint32_t)MINBASE + ((d[j] - dmin) >> dsh)
                                    : (uint32_t)MINBASE + ((uint32_t)(ub0 + ustep * j) >> ush) + lane_sub;
        const uint32_t key = __umulhi(hx - b0, scale);  // < MINBASE, non-decreasing in x
        uint32_t b = sel_if_eq_f64(v[j], smin, minb, (uint32_t)(MINBASE - 1) - key);
        b = u < U ? b : (uint32_t)NB;
        ws[j] = b;
        old[j] = atomicAdd(&cnt[b], 1u);
      }
    }
    bool bigl = false;
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      if (j < rows) {
        bigl |= (old[j] >= (uint32_t)kJsBucketMax) & (ws[j] < (uint32_t)NB);
        ws[j] |= old[j] << 16;
      }
    }
    return bigl;
  };
  // count with delta = range / 2^shift: -1 = a range the key cannot take (the
  // pair is marked), else whether some bucket exceeds kJsBucketMax
  auto count = [&](const BsKey& kp) -> int {
    if (!kp.ok) return -1;  // uniform
    const double c = rfl_f64(kp.c), delta = kp.delta;
    const uint32_t b0 = __builtin_amdgcn_readfirstlane(kp.b0);
    const uint32_t scale = __builtin_amdgcn_readfirstlane(kp.scale);
    const bool cform = kp.cform != 0;
    const bool bigl = cform ? count_rows(std::true_type{}, c, delta, b0, scale)
                            : count_rows(std::false_type{}, c, delta, b0, scale);
    {
      const bool wbig = ballot(bigl) != 0ull;
      if (lane == 0) sm.big[wid] = wbig ? 1u : 0u;
    }
    __syncthreads();
    bool anybig = false;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) anybig |= sm.big[w] != 0u;
    return anybig ? 1 : 0;
  };
  int cs = count(sm.key);
  if (cs == 1) {  // uniform: every wave has read the flags; zero the counters, recount
    __syncthreads();
    uint4* c4 = (uint4*)cnt;
    for (int i = tid; i < NB / 4; i += BLOCK) c4[i] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    cs = count(bs_key_params<MINBASE, BYDOC>(smin, smax, nan, QF_BS_RETRY_SHIFT));
  }
  if (cs != 0) {  // uniform: a range the key cannot take, or a bucket still too big
    if (tid == 0) perm_put(p, po, kJsUnsorted);
    return true;
  }

  // ---- exclusive scan of the counters -> u16 starts in bk ----------------------------
  {
    constexpr int kPer = NB / BLOCK;  // counters per thread
    static_assert(kPer == 8 || kPer == 4, "one or two uint4 counter loads per thread");
    uint32_t c[kPer];
    if constexpr (kPer == 8) {
      const uint4 c0 = ((const uint4*)cnt)[tid * 2], c1 = ((const uint4*)cnt)[tid * 2 + 1];
      c[0] = c0.x; c[1] = c0.y; c[2] = c0.z; c[3] = c0.w;
      c[4] = c1.x; c[5] = c1.y; c[6] = c1.z; c[7] = c1.w;
    } else {  // (1,024 threads: join_learned_kernel)
      const uint4 c0 = ((const uint4*)cnt)[tid];
      c[0] = c0.x; c[1] = c0.y; c[2] = c0.z; c[3] = c0.w;
    }
    uint32_t tot = 0u;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const uint32_t x = c[i];
      c[i] = tot;
      tot += x;
    }
    const uint32_t incl = wave_incl_scan_dpp(tot);
    if (lane == 63) sm.wtot[wid] = incl;
    __syncthreads();  // also: every counter read before the scatter overwrites them
    uint32_t pre = incl - tot;
#pragma unroll
    for (int w = 0; w < WAVES - 1; ++w) pre += w < wid ? sm.wtot[w] : 0u;
    if constexpr (kPer == 8)
      ((uint4*)bk)[tid] = make_uint4((pre + c[0]) | ((pre + c[1]) << 16),
                                     (pre + c[2]) | ((pre + c[3]) << 16),
                                     (pre + c[4]) | ((pre + c[5]) << 16),
                                     (pre + c[6]) | ((pre + c[7]) << 16));
    else
      ((uint2*)bk)[tid] = make_uint2((pre + c[0]) | ((pre + c[1]) << 16),
                                     (pre + c[2]) | ((pre + c[3]) << 16));
    if (tid == 0) bk[NB] = (uint16_t)U;
  }
  __syncthreads();

  const bool nonneg = smin >= 0.0;  // block-uniform (smin folds -0.0 into +0.0)
  // ---- scatter: the value by position; u, bucket size and arrival kept ------------------
  uint32_t pa[ROWS], pw[ROWS];  // position; u << 16 | size << 8 | arrival
#pragma unroll
  for (int j = 0; j < ROWS; ++j) {
    const int u = ub0 + j * ustep + lane;
    if (j < rows && u < U) {
      const uint32_t b = ws[j] & 0xFFFFu, at = ws[j] >> 16;
      const uint32_t st = bk[b], nx = bk[b + 1];
      const uint32_t pos = st + at;
      // the rank phase compares integer keys: for a pair without negative scores
      // (every C2 fusion) the f64 bits of v + 0.0 (-0.0 folded) already ascend
      skey[pos] = nonneg ? (uint64_t)__double_as_longlong(v[j] + 0.0) : bs_rank_key(v[j]);
      if (BYDOC) sd[pos] = d[j];
      pa[j] = pos;
      pw[j] = ((uint32_t)u << 16) | ((nx - st) << 8) | at;  // size <= kJsBucketMax
    }
  }
  __syncthreads();  // the starts are dead: the u | size | arrival words over them
#pragma unroll
  for (int j = 0; j < ROWS; ++j) {
    const int u = ub0 + j * ustep + lane;
    if (j < rows && u < U) sw[pa[j]] = pw[j];
  }
  __syncthreads();

  // ---- rank inside the bucket, in position order --------------------------------------
  uint32_t P[ROWS], uo[ROWS];
#pragma unroll
  for (int j = 0; j < ROWS; ++j) {
    const int i = pbase + j * 64 + lane;
    P[j] = 0u;
    uo[j] = 0u;
    if (j < rows && i < U) {
      const uint64_t ki = skey[i];
      const uint32_t wi = sw[i];
      // the tie-break key: the whole word, whose top bits are u — distinct, so the
      // word order is the first-seen order — or, BYDOC, the docid
      const uint32_t ti = BYDOC ? sd[i] : wi;
      const uint32_t lo = (uint32_t)i - (wi & 0xFFu), hi = lo + ((wi >> 8) & 0xFFu);
      uint32_t before = 0u;
      // the bucket's members by pointer (two per step; a bucket of one: nothing to
      // count): no index arithmetic inside the loop
      const uint32_t k0 = hi - lo > 1u ? lo : hi;
      const uint64_t* pv = skey + k0;
      const uint64_t* const pend = skey + hi;
      const uint64_t* const plast = pend - 1;  // a pair remains while pv < plast
      const uint32_t* tp = BYDOC ? sd + k0 : sw + k0;
      for (; pv < plast; pv += 2, tp += 2) {
        // two ds_read_b64 (2 LDS cycles each) rather than the ds_read2_b64 the
        // compiler would merge them into (8 cycles: it serves 16 lanes at a time)
        const uint64_t v0 = pv[0];
        asm volatile("" ::: "memory");
        const uint64_t v1 = pv[1];
        const uint32_t t0 = tp[0], t1 = tp[1];
        before = add_if_precedes(before, ki, ti, v0, t0);
        before = add_if_precedes(before, ki, ti, v1, t1);
      }
      if (pv < pend) before = add_if_precedes(before, ki, ti, pv[0], tp[0]);
      P[j] = lo + before;
      uo[j] = wi >> 16;
    }
  }
  // ---- outputs (every row's position before any store) ----------------------------------
#pragma unroll
  for (int j = 0; j < ROWS; ++j) {
    const int i = pbase + j * 64 + lane;
    if (j < rows && i < U) perm_put(p, po + P[j], uo[j]);
  }
  return false;
}

// UMAX < kJsUMax with INLINE_FB (small unions, one wave: C1): a pair the bucket sort
// cannot order is sorted by the LSD window sort in the same workgroup (sort_one over
// the same LDS), so no fallback pass follows the launch.  Its registers are capped for
// seven waves per SIMD (72 VGPRs; a few spill): C1's 6,904 pair waves then fit the
// GPU's 7,168 slots (six per SIMD, unspilled: 0.0439-0.0473 against 0.0426-0.0429 ms
// per C1 step).
template <int BLOCK, int BITS, bool BYDOC, int UMAX = kJsUMax, bool INLINE_FB = false>
__global__ __launch_bounds__(BLOCK, BYDOC ? 6 : INLINE_FB ? 7 : 8) void bsort_kernel(FuseParams p) {
  constexpr int WAVES = BLOCK / 64, ROWS = (UMAX + BLOCK - 1) / BLOCK;
  using FbC = SortCfg<BLOCK, ROWS, 8>;
  constexpr int kBs = BsLds<BITS, BYDOC, UMAX, BLOCK>::kBytes;
  constexpr int kLds = INLINE_FB && (int)sizeof(SortShared<FbC>) > kBs ? (int)sizeof(SortShared<FbC>)
                                                                        : kBs;
  __shared__ __attribute__((aligned(16))) unsigned char lds[kLds];
  __shared__ BsShared<WAVES> sm;
  // wid is wave-uniform: readfirstlane puts it (and every row base derived from
  // it) in SGPRs, so the per-row address arithmetic is scalar
  const int tid = threadIdx.x, lane = tid & 63,
            wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  // BYDOC: one workgroup per query for the learned slot only
  const int M = BYDOC ? 1 : __popc(p.methods);
  const int64_t bid = block_id();
  const int64_t grp8 = bid >> 3, ngroups = (p.n_queries + 7) / 8;
  if (grp8 >= ngroups * M) return;  // a 2-D grid's padding workgroups (grid_for)
  // groups of 8 queries (query q on XCD q % 8, where the join wrote it), in
  // reverse: the join's last-written scores are the likeliest still cached.
  // grp8 / M by a scalar multiply-high (M <= 9: exact below 2^20 groups), not the
  // compiler's VALU division sequence
  int64_t gq;
  if (M == 1) {
    gq = grp8;
  } else if (grp8 < (1 << 20)) {  // M in [2, 9]: magic = ceil(2^32 / M) fits 32 bits
    const uint32_t magic = 0xFFFFFFFFu / (uint32_t)M + 1u;
    gq = (int64_t)__umulhi((uint32_t)grp8, magic);
  } else {
    gq = grp8 / M;
  }
  const int64_t q = (ngroups - 1 - gq) * 8 + (bid & 7);
  const int ms = BYDOC ? __popc(p.methods & (QF_LEARNED - 1)) : (int)(grp8 - gq * M);
  if (!BYDOC && (p.methods & QF_LEARNED) && ms == __popc(p.methods & (QF_LEARNED - 1))) return;
  if (q >= p.n_queries) return;
  const int U = p.union_count[q];
  const int64_t base = p.list_off[q * p.R];
  if (U < 1 || U > UMAX) return;  // error / fuse_large_kernel's
  double* io = p.fused + (int64_t)ms * p.out_stride + base;
  const int64_t po = (int64_t)ms * p.out_stride + base;  // perm of this pair
  const int rows = (U + BLOCK - 1) / BLOCK;
  const int wbase = wid * rows * 64;  // this wave's items: [wbase, wbase + rows * 64)
  double v[ROWS];
  uint32_t d[BYDOC ? ROWS : 1];
#pragma unroll
  for (int j = 0; j < ROWS; ++j) {  // every row's load in flight before the first use
    const int u = wbase + j * 64 + lane;
    // every row loads, past U a clamped duplicate (bsort_core masks the items past
    // U itself: no exec-mask branch around the loads), non-temporal: the scores
    // are read this once (round 4: 1.5-2 us of the sort)
    const uint32_t uc = min((uint32_t)u, (uint32_t)(U - 1));
    v[j] = __builtin_nontemporal_load(&io[uc]);
    if (BYDOC) d[j] = p.union_docid[base + uc];
  }
  const bool marked = bsort_core<BLOCK, BITS, BYDOC, UMAX>(p, lds, sm, v, d, U, wbase, 64, po);
  if constexpr (INLINE_FB) {
    if (marked) {  // uniform
      __syncthreads();
      sort_one<FbC>(p, *reinterpret_cast<SortShared<FbC>*>(lds), ms, U, base, false);
    }
  }
}

// ============================================================================
// bsort_fast_kernel (round 5) — the default path's sort of every non-learned slot
// with U <= UMAX: bsort_kernel's bucket sort (same order: scores descending, ties in
// first-seen u order) with fewer instructions per item; bsort_kernel keeps learned
// fusion's docid-tie slot (BYDOC) and C1's one-wave form.
//  * key constants from the join (pair_info: the slot's min / max and the key's
//    constants at fused[slot][base + U]) — no range phase, no block reduction, no
//    serial wave-0 section; computed here only when the join left none;
//  * the scores read with buffer loads: one voffset for every row (the row offset in
//    the instruction), the hardware returns 0.0 past U — no clamp, no per-row address;
//  * bucket = mul_hi(top - hi32(x), scale): larger scores first without a subtraction;
//    lanes past U count into spare counters (NB + lane % 16, < 64 arrivals each), so
//    a bucket overflow is one running max of the arrival indices, read after the
//    count's barrier;
//  * the rank walks its bucket including itself (a member never precedes itself): no
//    singleton select, bucket bounds from the word (u << 16 | size << 8 | arrival);
//  * perm written with buffer stores (one shift per row).
// LDS: region A = the keys by position (u64 [UMAX]; before the scatter, the u32
// counters), region B = the words by position (u32 [UMAX]; before them, the u16
// bucket starts).  UMAX 3,072 with 512 threads: 36 KB, 4 workgroups per CU.
// ============================================================================
constexpr int kFastSpare = 16;  // counters of the lanes past U
template <int UMAX, int BITS, bool S32>
struct BsFastLds {
  static constexpr int kNB = 1 << BITS;
  // one position more than UMAX: the sentinel at position U (see the rank phase);
  // S32: u32 bucket starts (one ds_read2_b32 for a bucket's start and end)
  static constexpr int kA = 8 * (UMAX + 2);
  static constexpr int kStarts = (S32 ? 4 : 2) * (kNB + 8);
  static constexpr int kB = 4 * (UMAX + 2) > kStarts ? 4 * (UMAX + 2) : kStarts;
  static constexpr int kBytes = kA + kB;
  static_assert(4 * (kNB + kFastSpare) <= kA, "counters in region A");
};
template <int WAVES>
struct BsFastShared {
  uint32_t wtot[WAVES];
  double mn[WAVES], mx[WAVES];  // the in-kernel range (no constants from the join)
  uint32_t big, nan;
};

// one 16-byte LDS store: the compiler splits a uint4 store whose registers it did
// not allocate as an aligned tuple into b96 + write2 + b32 stores, which at the
// scan's 32-byte lane stride conflict eight ways (round 5: 53 us of the 1,024-thread
// configuration's 332; two-way as one b128)
typedef unsigned int qf_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void lds_store_b128(void* at, uint32_t a, uint32_t b, uint32_t c,
                                               uint32_t d) {
  const uint32_t addr = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)at;
  const qf_u32x4 v = {a, b, c, d};
  asm volatile("ds_write_b128 %0, %1" ::"v"(addr), "v"(v) : "memory");
}

// UMIN < U <= UMAX of the pairs this configuration sorts; BITS: 2^BITS buckets (the
// last 1/16 the minimum's sub-buckets); S32: u32 bucket starts.
template <int BLOCK, int UMIN, int UMAX, int BITS, bool S32, int MINW>
__global__ __launch_bounds__(BLOCK, MINW) void bsort_fast_kernel(FuseParams p) {
  constexpr int WAVES = BLOCK / 64, ROWS = UMAX / BLOCK, NB = 1 << BITS;
  constexpr int MINSUB = NB / 16, MINBASE = NB - MINSUB;
  static_assert(ROWS * BLOCK == UMAX && UMAX <= 65535, "rows of a wave");
  static_assert(((UMAX - 1) >> 6) < MINSUB, "minimum sub-bucket shift <= 6");
  static_assert(NB % (4 * BLOCK) == 0, "whole uint4 counter loads per thread");
  using LD = BsFastLds<UMAX, BITS, S32>;
  __shared__ __attribute__((aligned(16))) unsigned char lds[LD::kBytes];
  __shared__ BsFastShared<WAVES> sm;
  uint64_t* skey = (uint64_t*)lds;               // region A from the scatter on
  uint32_t* cnt = (uint32_t*)lds;                // region A until the scan
  uint32_t* sw = (uint32_t*)(lds + LD::kA);      // region B from the second scatter on
  uint16_t* bk = (uint16_t*)(lds + LD::kA);      // region B until then (u16 starts)
  uint32_t* bk32 = (uint32_t*)(lds + LD::kA);    // (S32: u32 starts)
  const int tid = threadIdx.x, lane = tid & 63,
            wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = __popc(p.methods);
  const int64_t bid = block_id();
  const int64_t grp8 = bid >> 3, ngroups = (p.n_queries + 7) / 8;
  if (grp8 >= ngroups * M) return;
  // groups of 8 queries (query q on XCD q % 8, where the join wrote it), in reverse
  // (the join's last-written scores are the likeliest still cached); grp8 / M by a
  // scalar multiply-high (exact below 2^20 groups)
  int64_t gq;
  if (M == 1) gq = grp8;
  else if (grp8 < (1 << 20)) gq = (int64_t)__umulhi((uint32_t)grp8, 0xFFFFFFFFu / (uint32_t)M + 1u);
  else gq = grp8 / M;
  const int64_t q = (ngroups - 1 - gq) * 8 + (bid & 7);
  const int ms = (int)(grp8 - gq * M);
  if ((p.methods & QF_LEARNED) && ms == __popc(p.methods & (QF_LEARNED - 1))) return;
  if (q >= p.n_queries) return;
  // the three loads in flight together (the offsets before the range check: one
  // memory latency, not two, before the scores' loads can issue)
  const int U = p.union_count[q];
  const int64_t base = p.list_off[q * p.R];
  const int64_t nq = p.list_off[q * p.R + p.R] - base;
  if (U < 1 || U <= UMIN || U > UMAX) return;  // a status, or another kernel's
  const double* io = p.fused + (int64_t)ms * p.out_stride + base;
  const int64_t po = (int64_t)ms * p.out_stride + base;
  const int rows = (U + BLOCK - 1) / BLOCK;
  const int wbase = wid * rows * 64;  // this wave's items / positions: [wbase, wbase + rows * 64)

  // ---- loads (past U: 0.0, masked below) --------------------------------------------
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)io, (short)0, U * 8, 0x00020000);
  const int voff = (wbase + lane) * 8;
  double v[ROWS];
#pragma unroll
  for (int j = 0; j < ROWS; ++j)
    if (j < rows)  // uniform
      v[j] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, voff + j * 512, 0,
                                                                             kBufNT));
  // the counters zeroed while the loads are in flight
  for (int i = tid; i < (NB + kFastSpare) / 4; i += BLOCK)
    ((uint4*)cnt)[i] = make_uint4(0u, 0u, 0u, 0u);
  if (tid == 0) {
    sm.big = 0u;
    sm.nan = 0u;
  }
  // ---- the key constants: the join's, else computed here ------------------------------
  double smin = 0.0, smax = 0.0, kc = 0.0;
  uint64_t w3 = 0ull;
  if (nq - U >= kPairInfo) {  // uniform
    const double* inf = io + U;
    smin = rfl_f64(inf[0]);
    smax = rfl_f64(inf[1]);
    kc = rfl_f64(inf[2]);
    const uint64_t w = ((const uint64_t*)inf)[3];
    w3 = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(w >> 32)) << 32) |
         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)w);
  }
  __syncthreads();  // the counters and flags are zero
  if (w3 == 0ull) {  // uniform: the range of the valid items, reduced over the block
    double vmn = INFINITY, vmx = -INFINITY;
    bool nan = false;
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      const int u = wbase + j * 64 + lane;
      if (j < rows && u < U) {
        vmn = raw_min_f64(vmn, v[j]);
        vmx = raw_max_f64(vmx, v[j]);
        nan |= v[j] != v[j];
      }
    }
    vmn = wave_min_f64_dpp(vmn);
    vmx = wave_max_f64_dpp(vmx);
    if (ballot(nan) != 0ull && lane == 0) sm.nan = 1u;
    if (lane == 63) {
      sm.mn[wid] = vmn;
      sm.mx[wid] = vmx;
    }
    __syncthreads();
    double a = sm.mn[0], b = sm.mx[0];
#pragma unroll
    for (int w = 1; w < WAVES; ++w) {
      a = raw_min_f64(a, sm.mn[w]);
      b = raw_max_f64(b, sm.mx[w]);
    }
    smin = rfl_f64(a + 0.0);
    smax = rfl_f64(b + 0.0);
    const bool anynan = sm.nan != 0u;
    if (anynan) smin = smax = __longlong_as_double(0x7FF8000000000000ll);  // never "all equal"
    const BsKey2 k = bs_key2<MINBASE>(smin, smax, anynan, kFastDeltaShift);
    kc = rfl_f64(k.c);
    const uint64_t w = bs_key2_word(k);
    w3 = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(w >> 32)) << 32) |
         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)w);
  }
  if (smin == smax) {  // every score equal: first-seen order
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      const int u = wbase + j * 64 + lane;
      if (j < rows && u < U) perm_put(p, po + u, (uint32_t)u);
    }
    return;
  }
  if (w3 == kPairMark) {  // a range the key cannot take: the fallback pass
    if (tid == 0) perm_put(p, po, kJsUnsorted);
    return;
  }
  QF_STOP(21, [&] { uint32_t a = 0u; for (int j = 0; j < ROWS; ++j) a += (uint32_t)__double2loint(v[j]); return a; },
          if (_qf_acc == 12345u) perm_put(p, po, 0u); return;);

  // ---- count --------------------------------------------------------------------------
  int ush = 0;  // (U - 1) >> ush < MINSUB: the minimum's sub-bucket is MINBASE + (u >> ush)
  while (((uint32_t)(U - 1) >> ush) >= (uint32_t)MINSUB) ++ush;
  const uint32_t lane_sub = (uint32_t)lane >> ush;  // (64-aligned row bases: exact split)
  const uint32_t spare = (uint32_t)NB + ((uint32_t)lane & (kFastSpare - 1u));
  uint32_t ws[ROWS];  // bucket | arrival << 16
  uint32_t omax = 0u;
  auto count_rows = [&](auto cf, double c, uint32_t top, uint32_t scale) __attribute__((always_inline)) {
    constexpr bool CF = decltype(cf)::value;
    uint32_t old[ROWS];
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      if (j < rows) {  // uniform; every row's atomic issued before any result is used
        const int u = wbase + j * 64 + lane;
        const double x = CF ? v[j] + c : (v[j] - smin) + c;
        const uint32_t hx = (uint32_t)((uint64_t)__double_as_longlong(x) >> 32);
        const uint32_t key = __umulhi(top - hx, scale);  // < MINBASE, 0 for the largest
        const uint32_t minb = ((uint32_t)MINBASE + ((uint32_t)(wbase + 64 * j) >> ush)) + lane_sub;
        uint32_t b = sel_if_eq_f64(v[j], smin, minb, key);
        b = u < U ? b : spare;
        ws[j] = b;
        old[j] = atomicAdd(&cnt[b], 1u);
      }
    }
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      if (j < rows) {
        omax = max(omax, old[j]);
        ws[j] |= old[j] << 16;
      }
    }
  };
  auto count = [&](double c, uint64_t w) __attribute__((always_inline)) {
    const uint32_t top = (uint32_t)w & 0x7FFFFFFFu, scale = (uint32_t)(w >> 32);
    if ((w >> 31) & 1u) count_rows(std::true_type{}, c, top, scale);
    else count_rows(std::false_type{}, c, top, scale);
    if (omax >= (uint32_t)kJsBucketMax) sm.big = 1u;  // (benign race: every writer stores 1)
  };
  count(kc, w3);
  __syncthreads();  // the counters are complete
  if (sm.big) {  // uniform, rare: recount with delta = range / 2^20
    __syncthreads();  // every thread has read the flag
    for (int i = tid; i < (NB + kFastSpare) / 4; i += BLOCK)
      ((uint4*)cnt)[i] = make_uint4(0u, 0u, 0u, 0u);
    if (tid == 0) sm.big = 0u;
    const BsKey2 k = bs_key2<MINBASE>(smin, smax, false, kFastRetryShift);
    __syncthreads();
    if (!k.ok) {  // uniform
      if (tid == 0) perm_put(p, po, kJsUnsorted);
      return;
    }
    omax = 0u;
    const uint64_t w = bs_key2_word(k);
    count(rfl_f64(k.c), ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(w >> 32)) << 32) |
                            (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)w));
    __syncthreads();
    if (sm.big) {  // uniform: still a bucket above kJsBucketMax — the fallback pass
      if (tid == 0) perm_put(p, po, kJsUnsorted);
      return;
    }
  }
  QF_STOP(22, [&] { uint32_t a = 0u; for (int j = 0; j < ROWS; ++j) a += ws[j]; return a; },
          if (_qf_acc == 12345u) perm_put(p, po, 0u); return;);

  // ---- exclusive scan of the counters -> u16 bucket starts (region B) ------------------
  {
    constexpr int kPer = NB / BLOCK;  // 8 (512 threads) or 4 (1,024)
    uint32_t c[kPer];
#pragma unroll
    for (int i = 0; i < kPer / 4; ++i) {
      const uint4 x = ((const uint4*)cnt)[tid * (kPer / 4) + i];
      c[4 * i] = x.x; c[4 * i + 1] = x.y; c[4 * i + 2] = x.z; c[4 * i + 3] = x.w;
    }
    uint32_t tot = 0u;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const uint32_t x = c[i];
      c[i] = tot;
      tot += x;
    }
    const uint32_t incl = wave_incl_scan_dpp(tot);
    if (lane == 63) sm.wtot[wid] = incl;
    __syncthreads();  // also: every counter read before the scatter overwrites them
    // the waves before this one: lane w reads wave w's total (one LDS read, not a
    // serial loop of up to 15 dependent ones), a DPP scan, the lane wid - 1 of it
    uint32_t pre = incl - tot;
    const uint32_t wt = wave_incl_scan_dpp(lane < WAVES ? sm.wtot[lane] : 0u);
    if (wid > 0) pre += readlane_u32(wt, wid - 1);
    if constexpr (S32) {
#pragma unroll
      for (int i = 0; i < kPer / 4; ++i)
        lds_store_b128(&bk32[(tid * (kPer / 4) + i) * 4], pre + c[4 * i], pre + c[4 * i + 1],
                       pre + c[4 * i + 2], pre + c[4 * i + 3]);
      if (tid == 0) bk32[NB] = (uint32_t)U;
    } else {
      const uint32_t pre2 = pre * 0x10001u;  // (starts <= U < 2^16: no carry between halves)
      uint32_t pk[kPer / 2];
#pragma unroll
      for (int i = 0; i < kPer / 2; ++i) pk[i] = (c[2 * i] | (c[2 * i + 1] << 16)) + pre2;
      if constexpr (kPer >= 8) {
#pragma unroll
        for (int i = 0; i < kPer / 8; ++i)
          lds_store_b128(&bk[(tid * (kPer / 8) + i) * 8], pk[4 * i], pk[4 * i + 1], pk[4 * i + 2],
                         pk[4 * i + 3]);
      } else {
        ((uint2*)bk)[tid] = make_uint2(pk[0], pk[1]);
      }
      if (tid == 0) bk[NB] = (uint16_t)U;
    }
  }
  __syncthreads();
  QF_STOP(23, [&] { uint32_t a = 0u; for (int j = 0; j < ROWS; ++j) a += ws[j] + bk[j]; return a; },
          if (_qf_acc == 12345u) perm_put(p, po, 0u); return;);

  // ---- scatter: keys by position, then the words over the dead starts ---------------
  uint32_t pa[ROWS], pw[ROWS];  // position; u << 16 | size << 8 | arrival
  const uint32_t ul = (uint32_t)(wbase + lane) << 16;
  auto scatter = [&](auto nn) __attribute__((always_inline)) {
    constexpr bool NN = decltype(nn)::value;
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      const int u = wbase + j * 64 + lane;
      if (j < rows && u < U) {
        const uint32_t b = ws[j] & 0xFFFFu, at = ws[j] >> 16;
        const uint32_t st = S32 ? bk32[b] : bk[b], nx = S32 ? bk32[b + 1] : bk[b + 1];
        const uint32_t pos = QF_DEV_SCATTER_POS(st + at, (uint32_t)u);
        // the rank phase compares integer keys: without negative scores (every C2
        // fusion) the f64 bits of v + 0.0 (-0.0 folded) already ascend
        skey[pos] = NN ? (uint64_t)__double_as_longlong(v[j] + 0.0) : bs_rank_key(v[j]);
        pa[j] = pos;
        pw[j] = (ul + ((uint32_t)(64 * j) << 16)) | ((nx - st) << 8) | at;
      }
    }
  };
  if (smin >= 0.0) scatter(std::true_type{});  // uniform
  else scatter(std::false_type{});
  __syncthreads();  // the starts are dead
#pragma unroll
  for (int j = 0; j < ROWS; ++j) {
    const int u = wbase + j * 64 + lane;
    if (j < rows && u < U) sw[pa[j]] = pw[j];
  }
  // a sentinel at position U (key 0 = the smallest, tie word ~0 = the largest: it
  // never precedes anything), so the rank loop may read one member past a bucket's
  // end — a later bucket's member never precedes either (later buckets hold strictly
  // smaller scores; the minimum's sub-buckets equal scores with larger u)
  if (tid == 0) {
    skey[U] = 0ull;
    sw[U] = 0xFFFFFFFFu;
  }
  __syncthreads();
  QF_STOP(24, [&] { uint32_t a = 0u; for (int j = 0; j < ROWS; ++j) a += pa[j] + sw[j]; return a; },
          if (_qf_acc == 12345u) perm_put(p, po, 0u); return;);

  // ---- rank inside the bucket, in position order --------------------------------------
  // LDS byte offsets: keys at 8 * position, words at kA + 4 * position; this lane's
  // row j reads position wbase + lane + 64 j (the row part an instruction offset)
  uint32_t P[ROWS], uo[ROWS];
  const unsigned char* kme = lds + 8 * (wbase + lane);
  const unsigned char* wme = lds + LD::kA + 4 * (wbase + lane);
#pragma unroll
  for (int j = 0; j < ROWS; ++j) {
    const int i = wbase + j * 64 + lane;
    P[j] = 0u;
    uo[j] = 0u;
    if (j < rows && i < U) {
      const uint64_t ki = *(const uint64_t*)(kme + 512 * j);
      const uint32_t wi = *(const uint32_t*)(wme + 256 * j);  // also the tie-break key:
      // u in the top bits (distinct), so the word order is the first-seen order
      const uint32_t lo = (uint32_t)i - (wi & 0xFFu);
      uint32_t ka = lo * 8u;  // the bucket's first key
      asm volatile("" : "+v"(ka));  // (kept, not re-derived from i in the loop's preheader)
      const uint32_t kend = ka + __builtin_amdgcn_ubfe(wi, 8u, 8u) * 8u;  // one past its last
      uint32_t ta = LD::kA + lo * 4u;  // the first word
      uint32_t before = 0u;
      // every member, itself included (it never precedes itself), two per step; an odd
      // bucket's last step reads the member after it, which never precedes (sentinel)
      do {  // (a bucket holds this position: at least one step)
        // two ds_read_b64 (2 LDS cycles each) rather than a ds_read2_b64 (8 cycles)
        const uint64_t v0 = *(const uint64_t*)(lds + ka);
        asm volatile("" ::: "memory");
        const uint64_t v1 = *(const uint64_t*)(lds + ka + 8);
        const uint32_t t0 = *(const uint32_t*)(lds + ta), t1 = *(const uint32_t*)(lds + ta + 4);
        before = add_if_precedes(before, ki, wi, v0, t0);
        before = add_if_precedes(before, ki, wi, v1, t1);
        ka += 16u;
        ta += 8u;
      } while (ka < kend);
      P[j] = lo + before;
      uo[j] = wi >> 16;
    }
  }
  QF_STOP(25, [&] { uint32_t a = 0u; for (int j = 0; j < ROWS; ++j) a += P[j] + uo[j]; return a; },
          if (_qf_acc == 12345u) perm_put(p, po, 0u); return;);
  // ---- perm (every row's position before any store) ------------------------------------
  if (p.perm32) {  // uniform
    const auto pr = __builtin_amdgcn_make_buffer_rsrc((uint32_t*)p.perm + po, (short)0, U * 4,
                                                      0x00020000);
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      const int i = wbase + j * 64 + lane;
      if (j < rows && i < U) __builtin_amdgcn_raw_buffer_store_b32(uo[j], pr, P[j] * 4, 0, kBufNT);
    }
  } else {
    const auto pr = __builtin_amdgcn_make_buffer_rsrc((uint16_t*)p.perm + po, (short)0, U * 2,
                                                      0x00020000);
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      const int i = wbase + j * 64 + lane;
      if (j < rows && i < U)
        __builtin_amdgcn_raw_buffer_store_b16((uint16_t)uo[j], pr, P[j] * 2, 0, kBufNT);
    }
  }
}

// ============================================================================
// join_learned_kernel — learned fusion alone (C5: QF_LEARNED is the call's one
// method), join and sort in one workgroup per query.  The LDS join as join_kernel
// (JoinM: N <= 5,120, micro-unit scores), then each thread's documents u = j *
// 512 + tid take pandas' Kahan sums (src/fusion.py:436-446) — stored as
// join_kernel stores them — and stay in registers with their docids (the group's
// first entry's input docid), and the bucket sort by docid ties (bsort_core,
// BYDOC) ranks them in the join's dead LDS.  The separate sort kernel re-read
// every score from HBM and ran at 3 workgroups per CU for the docid array;
// here the scores never leave the registers.  Unions up to kLearnedUMax = 4,608
// (SURVEY §8(d)'s C2 unions: 3,856-4,148): the sort's 72 KB of LDS (12-bit keys,
// docids by position) over the join's dead tables, two workgroups per CU.  A union
// above it (or a query with a status) is left unsorted to fuse_large_kernel, as
// the join_kernel path leaves it.
// ============================================================================
constexpr int kLearnedUMax = 4608;
template <class C>
__global__ __launch_bounds__(C::kBlock, C::kMinWaves) void join_learned_kernel(FuseParams p) {
  constexpr int BLOCK = C::kBlock, ROWS = (kLearnedUMax + BLOCK - 1) / BLOCK;
  static_assert(BLOCK == 512 || BLOCK == 1024, "bsort_core's configurations");
  constexpr int kSortLds = BsLds<12, true, kLearnedUMax, BLOCK>::kBytes;
  __shared__ JoinShared<C, 1, kSortLds> sh;
  __shared__ BsShared<BLOCK / 64> sm;
  const int64_t q = block_id();
  if (q >= p.n_queries) return;
  const int N = join_groups<C, 1, kSortLds>(p, sh, q);
  if (N < 0) return;
  const int U = sh.U;
  if (U > kLearnedUMax || sh.status) {  // uniform: the fallback pass's share
    SlotRange rg;  // (learned fusion alone keeps no ranges)
    store_unsorted_sums<C, 1, kSortLds>(p, sh, N, rg);
    if (threadIdx.x == 0) p.union_count[q] = sh.status ? sh.status : U;
    return;
  }
  using L = JoinLds<C, 1>;
  const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t base = sh.off[0];
  const int32_t* gsc = (const int32_t*)(sh.smem + L::kGscOff);
  const uint32_t* gpr = (const uint32_t*)(sh.smem + L::kGprOff);
  const uint16_t* ugo = (const uint16_t*)(sh.smem + L::kGoOff);
  double v[ROWS];
  uint32_t d[ROWS];
#pragma unroll
  for (int j = 0; j < ROWS; ++j) {
    const int u = j * BLOCK + tid;
    v[j] = 0.0;
    d[j] = 0u;
    if (u < U) {
      const int gs = ugo[u], ge = u + 1 < U ? (int)ugo[u + 1] : N;
      const uint32_t g0 = gpr[gs];  // the first-seen entry: the document's docid
      d[j] = p.docid[sh.off[g0 >> 16] + (g0 & 0xFFFFu)];
      double a6 = 0.0, c6 = 0.0;
      for (int k = gs; k < ge; ++k) {
        const double s = ScoreIn<1>::val(gsc[k]);
        const int r = (int)(gpr[k] >> 16);
        learned_add(p, s, sh.w[r], r, a6, c6);  // src/fusion.py:436-446
      }
      v[j] = a6;
      p.fused[base + u] = a6;  // the one method slot
    }
  }
  if (tid == 0) p.union_count[q] = U;
  QF_STOP(40, [&] { uint32_t a = 0u; for (int j = 0; j < ROWS; ++j) a += d[j] + (uint32_t)__double2loint(v[j]); return a; },
          if (_qf_acc == 12345u) p.union_count[q] = 0; return;);
  __syncthreads();  // the groups are dead: their LDS is the sort's
  bsort_core<BLOCK, 12, true, kLearnedUMax>(p, sh.smem, sm, v, d, U, wid * 64, BLOCK, base);
}

// ============================================================================
// join_sort_xl_kernel — queries beyond the LDS join (JoinXL::kNMax < N <= 65,535,
// e.g. 16 runs x top-4000): the same algorithm with its tables in a global
// workspace, one 1,024-thread workgroup per query.
//   1. insert every entry into a hash table (docid, retriever mask:
//      atomicCAS / atomicOr), remembering each entry's slot;
//   2. number documents u in first-seen order (a document's representative is
//      its entry in the lowest retriever holding it, as in the LDS join; block
//      scans over the entries in order);
//   3. group offsets (scan of the masks' popcounts), each entry's place in its
//      group in retriever order, and DocSums over every group — the same sums
//      as the LDS join, bit for bit;
//   4. unions of up to 10,240 documents are left unsorted, with their U, to the
//      LDS sort kernels launched after this one; larger ones get, per method
//      slot, the bucket sort of bsort_kernel over the workspace (xl_bsort:
//      16,384 buckets counted in LDS, scores and tie words scattered to the
//      workspace by bucket, each item ranked inside its bucket).  A slot it
//      cannot order (a bucket above kXlBucketMax after the finer recount, a
//      non-finite range, a NaN) takes a bitonic sort of (key = ~orderable(score),
//      tie = u — or docid for learned fusion) — unique pairs, so the order equals
//      the stable sort of the LDS path: passes with stride >= kXlTile run in the
//      workspace, the rest on kXlTile-item tiles in LDS.
// u and every entry index are 32-bit: up to kXlNMaxWide entries per query with
// qf_fuse_wide's uint32 perm (kXlNMax with qf_fuse's uint16 perm).
// A persistent grid of G <= 512 workgroups (two per CU) lists the large queries of each strided
// chunk (one parallel load of their sizes) and runs them in turn, so batches
// without large queries cost one short launch — and fuse_launch only makes it
// when max_entries says a large query may exist.
// ============================================================================
constexpr int kXlBlock = 1024;
constexpr int kXlTile = 4096;  // bitonic items per LDS tile (64 KB of keys + ties)
constexpr int kXlUnroll = 4;   // entries per thread per step of the join's phases
constexpr int kXlNMax = 65535;  // entries per query with a uint16 perm
constexpr int kXlNMaxWide = (1 << 24) - 1;  // with a uint32 perm (grouped entries: e | r << 27)
constexpr int kXlGrid = 512;   // workgroups: two per CU (75 KB of LDS each)

struct XlWs {
  uint32_t *tkey, *tmask, *tu;           // [TS] hash table
  uint32_t *eslot, *umask, *ugo, *gent;  // [NMAX] entry slot, document masks / group
                                         // starts, grouped entries (e | r << 27)
  uint64_t *skey, *stie;                 // [P] sort keys and ties (bitonic)
  double* sval;                          // [P] unsorted scores (bitonic); scores by
                                         // position (bucket sort)
  // the bucket sort's views of skey / stie: tie | size | arrival by position,
  // bucket | arrival by u, u by position (learned fusion)
  uint64_t* sw;
  uint32_t *sarr, *su;
};
static __host__ __device__ inline int64_t xl_ws_bytes(int ts, int nmax, int np) {
  const int64_t a = 12 * (int64_t)ts + 16 * (int64_t)nmax + 24 * (int64_t)np;
  return (a + 255) & ~(int64_t)255;
}
__device__ __forceinline__ XlWs xl_ws(unsigned char* b, int ts, int nmax, int np) {
  XlWs w;
  uint32_t* t = (uint32_t*)b;
  w.tkey = t; w.tmask = t + ts; w.tu = t + 2 * ts;
  uint32_t* e = t + 3 * ts;
  w.eslot = e; w.umask = e + nmax; w.ugo = e + 2 * nmax; w.gent = e + 3 * nmax;
  uint64_t* k = (uint64_t*)(((uintptr_t)(e + 4 * nmax) + 7) & ~(uintptr_t)7);
  w.skey = k; w.stie = k + np; w.sval = (double*)(k + 2 * np);
  w.sw = w.skey;
  w.sarr = (uint32_t*)w.stie;
  w.su = w.sarr + np;
  return w;
}

// Phase boundary of the workspace kernel.  One workgroup owns its workspace and
// its waves share one CU's write-through L1, so a workgroup barrier orders the
// plain stores; an agent-scope fence here (an L2 write-back on gfx950) made the
// kernel ~10x slower.  The L2 atomics of the hash table are read back with
// L1-bypassing atomic loads instead (xl_ld).
__device__ __forceinline__ void xl_sync() { __syncthreads(); }
__device__ __forceinline__ uint32_t xl_ld(const uint32_t* a) {
  return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Exclusive scan of v over the 1,024 threads; *total gets the sum.
__device__ __forceinline__ uint32_t xl_scan(uint32_t v, uint32_t* s_wsum, uint32_t* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t inc = wave_incl_scan_dpp(v);
  if (lane == 63) s_wsum[wid] = inc;
  __syncthreads();
  uint32_t before = 0, all = 0;
  for (int w = 0; w < kXlBlock / 64; ++w) {
    const uint32_t x = s_wsum[w];
    before += w < wid ? x : 0u;
    all += x;
  }
  __syncthreads();  // s_wsum is reused by the next call
  *total = all;
  return before + inc - v;
}

__device__ __forceinline__ void xl_cmpswap(uint64_t& ka, uint64_t& ta, uint64_t& kb,
                                           uint64_t& tb, bool asc) {
  const bool gt = ka > kb || (ka == kb && ta > tb);
  if (gt == asc) {
    const uint64_t k = ka, t = ta;
    ka = kb; ta = tb; kb = k; tb = t;
  }
}

// Bitonic stages on LDS tiles of T items: kk == 0 runs every stage k <= T in
// full; else stage kk from stride j0 down (the strides below T of a stage whose
// larger strides ran in the workspace).  Direction from the item's global index.
__device__ __forceinline__ void xl_tile_pass(uint64_t* __restrict__ gkey,
                                             uint64_t* __restrict__ gtie, uint64_t* t_key,
                                             uint64_t* t_tie, int NP, int T, int kk, int j0) {
  const int tid = threadIdx.x;
  for (int t0 = 0; t0 < NP; t0 += T) {
    for (int i = tid; i < T; i += kXlBlock) {
      t_key[i] = gkey[t0 + i];
      t_tie[i] = gtie[t0 + i];
    }
    __syncthreads();
    const int k_lo = kk ? kk : 2, k_hi = kk ? kk : T;
    for (int k2 = k_lo; k2 <= k_hi; k2 <<= 1) {
      for (int j = kk ? j0 : k2 >> 1; j > 0; j >>= 1) {
        for (int t = tid; t < T / 2; t += kXlBlock) {
          const int i = ((t & ~(j - 1)) << 1) | (t & (j - 1));
          uint64_t ka = t_key[i], ta = t_tie[i], kb = t_key[i + j], tb = t_tie[i + j];
          const bool asc = ((t0 + i) & k2) == 0;
          const bool gt = ka > kb || (ka == kb && ta > tb);
          if (gt == asc) {
            t_key[i] = kb; t_tie[i] = tb;
            t_key[i + j] = ka; t_tie[i + j] = ta;
          }
        }
        __syncthreads();
      }
    }
    for (int i = tid; i < T; i += kXlBlock) {
      gkey[t0 + i] = t_key[i];
      gtie[t0 + i] = t_tie[i];
    }
    __syncthreads();
  }
}

// ---- the workspace bucket sort of one (query, method slot) --------------------------
// bsort_kernel's algorithm with its per-item arrays in the workspace: 16,384
// u32 bucket counters in LDS (over the bitonic tiles), minimum's sub-buckets by u
// (BYDOC: by docid), a bucket above kXlBucketMax recounted once at the finer
// delta.  Returns false, perm untouched, for the bitonic fallback.
constexpr int kXlBits = 14, kXlNB = 1 << kXlBits;
constexpr int kXlMinSub = kXlNB / 16, kXlMinBase = kXlNB - kXlMinSub;
constexpr int kXlBucketMax = 256;
// delta = range / 2^10: four times bsort_kernel's buckets, two more binades
constexpr int kXlDeltaShift = 10;
struct XlScratch {  // the bucket sort's block reductions
  double mn[kXlBlock / 64], mx[kXlBlock / 64];
  uint32_t dmn[kXlBlock / 64], dmx[kXlBlock / 64];
  int flag[kXlBlock / 64];
};

template <bool BYDOC>
__device__ bool xl_bsort(const FuseParams& p, const double* __restrict__ io, int64_t base, int U,
                         int64_t po, const XlWs& w, uint32_t* cnt, uint32_t* s_wsum,
                         XlScratch* xs) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  constexpr int WAVES = kXlBlock / 64;
  // ---- score (and docid) range ---------------------------------------------------------
  double mn = INFINITY, mx = -INFINITY;
  uint32_t dmn = ~0u, dmx = 0u;
  int nan = 0;
  for (int u = tid; u < U; u += kXlBlock) {
    const double v = io[u];
    mn = raw_min_f64(mn, v);
    mx = raw_max_f64(mx, v);
    nan |= v != v;
    if (BYDOC) {
      const uint32_t d = p.union_docid[base + u];
      dmn = min(dmn, d);
      dmx = max(dmx, d);
    }
  }
  mn = wave_min(mn);
  mx = wave_max(mx);
  nan = ballot(nan != 0) != 0ull;
  if (BYDOC) {
    dmn = (uint32_t)wave_min_u64_dpp(dmn);
    dmx = (uint32_t)wave_max_u64_dpp(dmx);
  }
  if (lane == 63) {
    xs->mn[wid] = mn;
    xs->mx[wid] = mx;
    xs->dmn[wid] = dmn;
    xs->dmx[wid] = dmx;
    xs->flag[wid] = nan;
  }
  __syncthreads();
  for (int i = 0; i < WAVES; ++i) {
    mn = fmin(mn, xs->mn[i]);
    mx = fmax(mx, xs->mx[i]);
    dmn = min(dmn, xs->dmn[i]);
    dmx = max(dmx, xs->dmx[i]);
    nan |= xs->flag[i];
  }
  __syncthreads();  // xs is reused below
  // the folded extremes (-0.0 == +0.0)
  const double smin = f64_from_asc_key(f64_asc_key(mn)), smax = f64_from_asc_key(f64_asc_key(mx));
  if (!BYDOC && !nan && smin == smax) {  // every score equal: first-seen order
    for (int u = tid; u < U; u += kXlBlock) perm_put(p, po + u, (uint32_t)u);
    return true;
  }
  int ush = 0, dsh = 0;  // minimum's sub-bucket: u >> ush (BYDOC: d - dmin >> dsh)
  while (((uint32_t)(U - 1) >> ush) >= (uint32_t)kXlMinSub) ++ush;
  if (BYDOC)
    while (((dmx - dmn) >> dsh) >= (uint32_t)kXlMinSub) ++dsh;
  // ---- count: one LDS atomic per item; bucket | arrival << 16 by u ------------------------
  auto count = [&](const BsKey& kp) -> int {
    for (int i = tid; i <= kXlNB; i += kXlBlock) cnt[i] = 0u;
    __syncthreads();
    if (!kp.ok) return -1;  // uniform
    int big = 0;
    for (int u = tid; u < U; u += kXlBlock) {
      const double v = io[u];
      const double x = kp.cform ? v + kp.c : (v - smin) + kp.delta;
      const uint32_t hx = (uint32_t)((uint64_t)__double_as_longlong(x) >> 32);
      const uint32_t key = __umulhi(hx - kp.b0, kp.scale);  // < kXlMinBase
      uint32_t b;
      if (v == smin)
        b = (uint32_t)kXlMinBase +
            (BYDOC ? (p.union_docid[base + u] - dmn) >> dsh : (uint32_t)u >> ush);
      else
        b = (uint32_t)(kXlMinBase - 1) - key;
      const uint32_t at = atomicAdd(&cnt[b], 1u);
      big |= at >= (uint32_t)kXlBucketMax;
      w.sarr[u] = b | (min(at, 0xFFFFu) << 16);
    }
    const bool wbig = ballot(big != 0) != 0ull;
    if (lane == 0) xs->flag[wid] = wbig ? 1 : 0;
    __syncthreads();
    int any = 0;
    for (int i = 0; i < WAVES; ++i) any |= xs->flag[i];
    __syncthreads();  // the flags are read before the next count writes them
    return any;
  };
  int cs = count(bs_key_params<kXlMinBase, BYDOC>(smin, smax, nan, kXlDeltaShift));
  if (cs == 1) cs = count(bs_key_params<kXlMinBase, BYDOC>(smin, smax, nan, QF_BS_RETRY_SHIFT));
  if (cs != 0) return false;  // uniform
  // ---- exclusive scan of the counters, in place; cnt[kXlNB] = U ----------------------------
  {
    constexpr int kPer = kXlNB / kXlBlock;
    static_assert(kPer == 16, "four uint4 counter loads per thread");
    const uint4* c4 = (const uint4*)cnt + tid * 4;
    uint32_t c[kPer];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint4 x = c4[i];
      c[4 * i] = x.x; c[4 * i + 1] = x.y; c[4 * i + 2] = x.z; c[4 * i + 3] = x.w;
    }
    uint32_t tot = 0u;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const uint32_t x = c[i];
      c[i] = tot;
      tot += x;
    }
    uint32_t all;
    const uint32_t pre = xl_scan(tot, s_wsum, &all);  // barriers: every counter read first
#pragma unroll
    for (int i = 0; i < kPer; ++i) cnt[tid * kPer + i] = pre + c[i];
    if (tid == 0) cnt[kXlNB] = (uint32_t)U;
  }
  __syncthreads();
  // ---- scatter: score and tie | size | arrival by position ---------------------------------
  for (int u = tid; u < U; u += kXlBlock) {
    const uint32_t a = w.sarr[u], b = a & 0xFFFFu, at = a >> 16;
    const uint32_t st = cnt[b], nx = cnt[b + 1];
    const uint32_t pos = st + at;
    const uint32_t tie = BYDOC ? p.union_docid[base + u] : (uint32_t)u;
    w.sval[pos] = io[u];
    w.sw[pos] = ((uint64_t)tie << 32) | ((nx - st) << 16) | at;
    if (BYDOC) w.su[pos] = (uint32_t)u;
  }
  xl_sync();
  // ---- rank inside the bucket: (score descending, tie ascending) ----------------------------
  const uint32_t* tw = (const uint32_t*)w.sw;  // the tie: the high word of sw[k]
  for (int i = tid; i < U; i += kXlBlock) {
    const double vi = w.sval[i];
    const uint64_t wi = w.sw[i];
    const uint32_t at = (uint32_t)wi & 0xFFFFu, sz = ((uint32_t)wi >> 16) & 0xFFFFu;
    const uint32_t ti = (uint32_t)(wi >> 32);
    const uint32_t lo = (uint32_t)i - at;
    uint32_t before = 0u;
    for (uint32_t k = lo; k < lo + sz; ++k) {
      const double vk = w.sval[k];
      const uint32_t tk = tw[2 * k + 1];
      before += (uint32_t)((vk > vi) | ((vk == vi) & (tk < ti)));
    }
    perm_put(p, po + lo + before, BYDOC ? w.su[i] : ti);
  }
  // (Measured, not kept: these loops four items per thread with their loads first,
  // as the join's phases — the kernel's spills grow 42 -> 72 VGPRs and the six sorts
  // of 500 x 16 x top-4000 take 5.08-5.46 ms against 4.74-5.10.)
  xl_sync();  // the workspace is the next slot's
  return true;
}

// ---- the workspace join's insert, partitioned ------------------------------------
// A query's hash table in the workspace is far larger than the caches once 500
// workgroups run (one ~1 MB table each), so every atomicCAS / atomicOr of the
// global insert was a random HBM read-modify-write.  Instead: count the entries
// per hash partition (LDS counters), scatter them by partition (entry | retriever
// << 27, docid), then join each partition in an LDS table of kXlPartSlots slots
// and number its distinct documents compactly (c = running count over the
// partitions).  Outputs as the global insert's: eslot[e] = the document's index c
// and tmask[c] = its retriever mask, both < U — so the numbering and placement
// that follow read small arrays.  A partition above kXlPartMax entries returns
// false (nothing the global insert needs was written) and the global insert runs.
constexpr int kXlPartBits = 13, kXlPartSlots = 1 << kXlPartBits;  // 64 KB of LDS
constexpr int kXlPartAvg = 2048;  // entries per partition on average
constexpr int kXlPartMax = 6144;  // at most 3/4 of the slots
constexpr int kXlPartRows = kXlPartMax / kXlBlock;

template <int KIND>
__device__ bool xl_partition_insert(const FuseParams& p, const XlWs& w, int64_t base, int N,
                                    const int64_t* s_off, uint32_t* lds, uint32_t* s_wsum,
                                    XlScratch* xs, int* s_status) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  constexpr int WAVES = kXlBlock / 64;
  int pbits = 0;
  while (((int64_t)kXlPartAvg << pbits) < (int64_t)N) ++pbits;
  const int P = 1 << pbits;  // <= 8,192 counters (N <= 2^24): 32 KB of the 64 KB
  auto part_of = [&](uint32_t d) -> uint32_t {
    return pbits ? (d * 0x9E3779B1u) >> (32 - pbits) : 0u;
  };
  uint32_t* pcnt = lds;        // [P]: counts, then fill cursors
  uint32_t* pe = w.tkey;       // [N] entry | retriever << 27, by partition
  uint32_t* pd = w.tkey + N;   // [N] docid, by partition (the table holds >= 2 N)
  uint32_t* pstart = w.ugo;    // [P + 1] (free until the group offsets)
  for (int i = tid; i < P; i += kXlBlock) pcnt[i] = 0u;
  __syncthreads();
  // ---- A. count per partition; the list checks of the global insert ----------------
  int status = 0, r = 0;
  for (int e0 = tid; e0 < N; e0 += kXlUnroll * kXlBlock) {
    uint32_t d[kXlUnroll];
    int rr[kXlUnroll];
#pragma unroll
    for (int j = 0; j < kXlUnroll; ++j) {
      const int e = e0 + j * kXlBlock;
      d[j] = 0u;
      if (e < N) {
        while (base + e >= s_off[r + 1]) ++r;
        d[j] = p.docid[base + e];
      }
      rr[j] = r;
    }
#pragma unroll
    for (int j = 0; j < kXlUnroll; ++j) {
      const int e = e0 + j * kXlBlock;
      if (e < N) {
        const int64_t g = base + e;
        if (d[j] == kEmpty) status = QF_QSTATUS_BADDOC;
        atomicAdd(&pcnt[part_of(d[j])], 1u);
        if (g + 1 < s_off[rr[j] + 1]) {
          if ((p.methods & (QF_COMBSUM | QF_COMBMNZ | QF_RRF)) &&
              ScoreIn<KIND>::raw(p.score, g + 1) > ScoreIn<KIND>::raw(p.score, g))
            status = QF_QSTATUS_UNSORTED;
          if ((p.methods & QF_WRRF) && p.rank && p.rank[g + 1] < p.rank[g])
            status = QF_QSTATUS_RANKORDER;
        }
      }
    }
  }
  if (status) atomicMin(s_status, status);
  __syncthreads();
  if (*s_status) return true;  // uniform: the caller reports it
  // ---- B. partition starts (exclusive scan), the largest partition ------------------
  {
    const int per = (P + kXlBlock - 1) / kXlBlock;  // counters per thread (<= 8)
    const int c0 = tid * per;
    uint32_t tot = 0u, mx = 0u;
    for (int i = 0; i < per; ++i)
      if (c0 + i < P) {
        tot += pcnt[c0 + i];
        mx = max(mx, pcnt[c0 + i]);
      }
    uint32_t all;
    uint32_t o = xl_scan(tot, s_wsum, &all);  // barriers: every count read first
    for (int i = 0; i < per; ++i)
      if (c0 + i < P) {
        const uint32_t c = pcnt[c0 + i];
        pstart[c0 + i] = o;
        pcnt[c0 + i] = o;
        o += c;
      }
    if (tid == 0) pstart[P] = (uint32_t)N;
    const bool big = ballot(mx > (uint32_t)kXlPartMax) != 0ull;
    if (lane == 0) xs->flag[wid] = big ? 1 : 0;
    __syncthreads();
    int any = 0;
    for (int i = 0; i < WAVES; ++i) any |= xs->flag[i];
    if (any) return false;  // uniform
  }
  // ---- C. scatter the entries by partition --------------------------------------------
  r = 0;
  for (int e0 = tid; e0 < N; e0 += kXlUnroll * kXlBlock) {
    uint32_t d[kXlUnroll], pos[kXlUnroll];
    int rr[kXlUnroll];
#pragma unroll
    for (int j = 0; j < kXlUnroll; ++j) {
      const int e = e0 + j * kXlBlock;
      d[j] = 0u;
      if (e < N) {
        while (base + e >= s_off[r + 1]) ++r;
        d[j] = p.docid[base + e];
      }
      rr[j] = r;
    }
#pragma unroll
    for (int j = 0; j < kXlUnroll; ++j)
      pos[j] = e0 + j * kXlBlock < N ? atomicAdd(&pcnt[part_of(d[j])], 1u) : 0u;
#pragma unroll
    for (int j = 0; j < kXlUnroll; ++j) {
      const int e = e0 + j * kXlBlock;
      if (e < N) {
        pe[pos[j]] = (uint32_t)e | ((uint32_t)rr[j] << 27);
        pd[pos[j]] = d[j];
      }
    }
  }
  xl_sync();
  // ---- D. each partition: LDS hash join, compact document numbering ------------------------
  uint32_t* key = lds;                 // [kXlPartSlots]: docid, then the compact index
  uint32_t* msk = lds + kXlPartSlots;  // [kXlPartSlots]: retriever mask
  const int hshift = 32 - pbits - kXlPartBits;  // the hash bits below the partition's
  uint32_t cbase = 0u;
  int dup = 0;
  for (int pp = 0; pp < P; ++pp) {
    const uint32_t a = pstart[pp], b = pstart[pp + 1];
    for (int i = tid; i < kXlPartSlots / 4; i += kXlBlock) {
      ((uint4*)key)[i] = make_uint4(kEmpty, kEmpty, kEmpty, kEmpty);
      ((uint4*)msk)[i] = make_uint4(0u, 0u, 0u, 0u);
    }
    __syncthreads();
    uint32_t hh[kXlPartRows], ev[kXlPartRows], dv[kXlPartRows];
#pragma unroll
    for (int j = 0; j < kXlPartRows; ++j) {
      const uint32_t k = a + (uint32_t)(tid + j * kXlBlock);
      ev[j] = k < b ? pe[k] : 0xFFFFFFFFu;
      dv[j] = k < b ? pd[k] : kEmpty;
    }
#pragma unroll
    for (int j = 0; j < kXlPartRows; ++j) {
      if (ev[j] != 0xFFFFFFFFu) {
        uint32_t h = ((dv[j] * 0x9E3779B1u) >> hshift) & (kXlPartSlots - 1);
        while (true) {
          const uint32_t prev = atomicCAS(&key[h], kEmpty, dv[j]);
          if (prev == kEmpty || prev == dv[j]) break;
          h = (h + 1) & (kXlPartSlots - 1);
        }
        const uint32_t rj = ev[j] >> 27;
        const uint32_t old = atomicOr(&msk[h], 1u << rj);
        dup |= (old >> rj) & 1u;
        hh[j] = h;
      }
    }
    __syncthreads();
    // compact index of each occupied slot, in slot order
    constexpr int kPer = kXlPartSlots / kXlBlock;  // 8
    const int s0 = tid * kPer;
    uint32_t occ = 0u, n_occ = 0u;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const bool o = key[s0 + i] != kEmpty;
      occ |= (uint32_t)o << i;
      n_occ += o;
    }
    uint32_t all;
    uint32_t c = cbase + xl_scan(n_occ, s_wsum, &all);  // barriers: every key read first
#pragma unroll
    for (int i = 0; i < kPer; ++i)
      if ((occ >> i) & 1u) {
        w.tmask[c] = msk[s0 + i];
        key[s0 + i] = c++;
      }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kXlPartRows; ++j)
      if (ev[j] != 0xFFFFFFFFu) w.eslot[ev[j] & 0x7FFFFFFu] = key[hh[j]];
    cbase += all;
    __syncthreads();  // the table is the next partition's
  }
  if (dup) atomicMin(s_status, QF_QSTATUS_DUPDOC);
  xl_sync();
  return true;
}

template <int KIND>
__device__ __forceinline__ void xl_one(const FuseParams& p, int64_t q, const XlWs& w, int tb, int pb,
                       int sort_min, int64_t* s_off, double* s_w, double* s_min, double* s_den,
                       double* s_rden, uint32_t* s_wsum, int* s_status, uint64_t* t_key,
                       uint64_t* t_tie, XlScratch* xs) {
  const int tid = threadIdx.x;
  const int R = p.R, TS = 1 << tb;
  if (tid <= R) s_off[tid] = p.list_off[q * R + tid];
  if (tid == 0) *s_status = 0;
  __syncthreads();
  const int64_t base = s_off[0];
  const int N = (int)(s_off[R] - base);  // JoinXL::kNMax < N <= kXlNMax (the lister's test)
  if (tid < R) {  // as the LDS join
    const int64_t a = s_off[tid], b = s_off[tid + 1];
    s_w[tid] = list_weight(p, q, tid, b > a);
    double mx = 0.0, mn = 0.0;
    if (b > a) {
      mx = ScoreIn<KIND>::load(p.score, a);
      mn = ScoreIn<KIND>::load(p.score, b - 1);
    }
    s_min[tid] = mn;
    s_den[tid] = ranx_den(mx, mn);
    s_rden[tid] = 1.0 / s_den[tid];
  }
  __syncthreads();  // s_status
  // ---- 1. insert: partitioned, else (a partition too large) the global table --------
  if (!xl_partition_insert<KIND>(p, w, base, N, s_off, (uint32_t*)t_key, s_wsum, xs, s_status)) {
  for (int i = tid; i < TS; i += kXlBlock) {
    w.tkey[i] = kEmpty;
    w.tmask[i] = 0u;
  }
  xl_sync();
  // kXlUnroll entries per thread per step, each phase's loads / atomics for all of
  // them issued before any result is used: the L2 atomic round trips overlap
  // (one entry per step left every thread waiting on one chain at a time)
  int status = 0, r = 0;
  for (int e0 = tid; e0 < N; e0 += kXlUnroll * kXlBlock) {
    uint32_t d[kXlUnroll], h[kXlUnroll], prev[kXlUnroll], old[kXlUnroll];
    int rr[kXlUnroll];
#pragma unroll
    for (int j = 0; j < kXlUnroll; ++j) {
      const int e = e0 + j * kXlBlock;
      d[j] = 0u;
      if (e < N) {
        while (base + e >= s_off[r + 1]) ++r;
        d[j] = p.docid[base + e];
      }
      rr[j] = r;
    }
#pragma unroll
    for (int j = 0; j < kXlUnroll; ++j) {
      h[j] = (d[j] * 0x9E3779B1u) >> (32 - tb);
      if (e0 + j * kXlBlock < N) {
        if (d[j] == kEmpty) status = QF_QSTATUS_BADDOC;
        prev[j] = atomicCAS(&w.tkey[h[j]], kEmpty, d[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < kXlUnroll; ++j) {
      if (e0 + j * kXlBlock < N) {
        while (prev[j] != kEmpty && prev[j] != d[j]) {  // probe on
          h[j] = (h[j] + 1) & (TS - 1);
          prev[j] = atomicCAS(&w.tkey[h[j]], kEmpty, d[j]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kXlUnroll; ++j)
      old[j] = e0 + j * kXlBlock < N ? atomicOr(&w.tmask[h[j]], 1u << rr[j]) : 0u;
#pragma unroll
    for (int j = 0; j < kXlUnroll; ++j) {
      const int e = e0 + j * kXlBlock;
      if (e < N) {
        const int64_t g = base + e;
        if ((old[j] >> rr[j]) & 1u) status = QF_QSTATUS_DUPDOC;
        w.eslot[e] = h[j];
        if (g + 1 < s_off[rr[j] + 1]) {
          if ((p.methods & (QF_COMBSUM | QF_COMBMNZ | QF_RRF)) &&
              ScoreIn<KIND>::raw(p.score, g + 1) > ScoreIn<KIND>::raw(p.score, g))
            status = QF_QSTATUS_UNSORTED;
          if ((p.methods & QF_WRRF) && p.rank && p.rank[g + 1] < p.rank[g])
            status = QF_QSTATUS_RANKORDER;
        }
      }
    }
  }
  if (status) atomicMin(s_status, status);
  xl_sync();
  }
  if (*s_status) {  // uniform
    if (tid == 0) p.union_count[q] = *s_status;
    __syncthreads();
    return;
  }
  // ---- 2. first-seen numbering ---------------------------------------------------
  // chunks of kXlUnroll * kXlBlock entries, kXlUnroll consecutive ones per thread (in
  // entry order: thread t's precede thread t + 1's), one block scan per chunk
  uint32_t U = 0;
  int r = 0;
  for (int c0 = 0; c0 < N; c0 += kXlUnroll * kXlBlock) {
    const int eb = c0 + tid * kXlUnroll;
    uint32_t h[kXlUnroll], msk[kXlUnroll], d[kXlUnroll];
    int rr[kXlUnroll];
#pragma unroll
    for (int j = 0; j < kXlUnroll; ++j) {
      h[j] = 0u;
      d[j] = 0u;
      if (eb + j < N) {
        while (base + eb + j >= s_off[r + 1]) ++r;
        h[j] = w.eslot[eb + j];
        d[j] = p.docid[base + eb + j];
      }
      rr[j] = r;
    }
    uint32_t n_rep = 0u, is_rep = 0u;
#pragma unroll
    for (int j = 0; j < kXlUnroll; ++j) {
      msk[j] = eb + j < N ? xl_ld(&w.tmask[h[j]]) : 0u;
      const bool rp = eb + j < N && __ffs(msk[j]) - 1 == rr[j];
      is_rep |= (uint32_t)rp << j;
      n_rep += rp;
    }
    uint32_t tot;
    uint32_t u = U + xl_scan(n_rep, s_wsum, &tot);
#pragma unroll
    for (int j = 0; j < kXlUnroll; ++j) {
      if ((is_rep >> j) & 1u) {
        w.tu[h[j]] = u;
        w.umask[u] = msk[j];
        p.union_docid[base + u] = d[j];  // the entry's own docid (= the table's key)
        ++u;
      }
    }
    U += tot;
  }
  xl_sync();
  // ---- 3. groups and sums -------------------------------------------------------
  uint32_t go = 0;
  for (int c0 = 0; c0 < (int)U; c0 += kXlBlock) {
    const int u = c0 + tid;
    const uint32_t pc = u < (int)U ? (uint32_t)__popc(w.umask[u]) : 0u;
    uint32_t tot;
    const uint32_t x = go + xl_scan(pc, s_wsum, &tot);
    if (u < (int)U) w.ugo[u] = x;
    go += tot;
  }
  xl_sync();
  r = 0;
  for (int e0 = tid; e0 < N; e0 += kXlUnroll * kXlBlock) {
    uint32_t hs[kXlUnroll], u[kXlUnroll];
    int rr[kXlUnroll];
#pragma unroll
    for (int j = 0; j < kXlUnroll; ++j) {
      const int e = e0 + j * kXlBlock;
      hs[j] = 0u;
      if (e < N) {
        while (base + e >= s_off[r + 1]) ++r;
        hs[j] = w.eslot[e];
      }
      rr[j] = r;
    }
#pragma unroll
    for (int j = 0; j < kXlUnroll; ++j) u[j] = e0 + j * kXlBlock < N ? w.tu[hs[j]] : 0u;
#pragma unroll
    for (int j = 0; j < kXlUnroll; ++j) {
      const int e = e0 + j * kXlBlock;
      if (e < N) {
        const uint32_t k =
            w.ugo[u[j]] + (uint32_t)__popc(w.umask[u[j]] & ((1u << rr[j]) - 1u));
        w.gent[k] = (uint32_t)e | ((uint32_t)rr[j] << 27);
      }
    }
  }
  xl_sync();
  const int methods = p.methods;
  const ListConsts lc{s_off, s_w, s_min, s_den, s_rden};
  for (int u = tid; u < (int)U; u += kXlBlock) {
    const int gs = (int)w.ugo[u], ge = u + 1 < (int)U ? (int)w.ugo[u + 1] : N;
    DocSums acc;
    for (int k = gs; k < ge; ++k) {
      const uint32_t v = w.gent[k];
      const int e = (int)(v & 0x7FFFFFFu), rr = (int)(v >> 27);
      acc.add(p, methods, lc, ScoreIn<KIND>::load(p.score, base + e), rr,
              (int)(base + e - s_off[rr]));
    }
    acc.store(p, methods, (double)(ge - gs), base + u);
  }
  xl_sync();
  // ---- 4. sort every method slot (unions the LDS sorts cannot hold) ---------------
  if ((int)U <= sort_min) {  // uniform: the LDS sort kernels that follow take it
    if (tid == 0) p.union_count[q] = (int)U;
    __syncthreads();
    return;
  }
  const int NP = 1 << pb, T = NP < kXlTile ? NP : kXlTile;
  const int M = __popc(methods);
  for (int ms = 0; ms < M; ++ms) {
    const bool by_docid = slot_method(methods, ms) == 6;
    double* io = p.fused + (int64_t)ms * p.out_stride + base;
    const int64_t po = (int64_t)ms * p.out_stride + base;
    const bool done = by_docid
                          ? xl_bsort<true>(p, io, base, (int)U, po, w, (uint32_t*)t_key, s_wsum, xs)
                          : xl_bsort<false>(p, io, base, (int)U, po, w, (uint32_t*)t_key, s_wsum, xs);
    if (done) continue;  // uniform
    for (int i = tid; i < NP; i += kXlBlock) {
      uint64_t k = ~0ull, t = ~0ull;  // padding sorts last
      if (i < (int)U) {
        const double v = io[i];
        w.sval[i] = v;
        k = ~f64_asc_key(v);
        t = by_docid ? ((uint64_t)p.union_docid[base + i] << 32) | (uint64_t)i : (uint64_t)i;
      }
      w.skey[i] = k;
      w.stie[i] = t;
    }
    xl_sync();
    xl_tile_pass(w.skey, w.stie, t_key, t_tie, NP, T, 0, 0);  // every stage k <= T
    for (int kk = 2 * T; kk <= NP; kk <<= 1) {
      for (int j = kk >> 1; j >= T; j >>= 1) {
        for (int t = tid; t < NP / 2; t += kXlBlock) {
          const int i = ((t & ~(j - 1)) << 1) | (t & (j - 1));
          uint64_t ka = w.skey[i], ta = w.stie[i], kb = w.skey[i + j], tb2 = w.stie[i + j];
          xl_cmpswap(ka, ta, kb, tb2, (i & kk) == 0);
          w.skey[i] = ka; w.stie[i] = ta; w.skey[i + j] = kb; w.stie[i + j] = tb2;
        }
        xl_sync();
      }
      xl_tile_pass(w.skey, w.stie, t_key, t_tie, NP, T, kk, T >> 1);
    }
    for (int i = tid; i < (int)U; i += kXlBlock) {
      perm_put(p, po + i, (uint32_t)(w.stie[i] & 0xFFFFFFFFu));
    }
    xl_sync();
  }
  if (tid == 0) p.union_count[q] = (int)U;
  __syncthreads();
}

template <int KIND>
__global__ __launch_bounds__(kXlBlock, 8) void join_sort_xl_kernel(FuseParams p, int nmin,
                                                                unsigned char* ws, int64_t ws_each,
                                                                int nmax, int tb, int pb,
                                                                int sort_min) {
  __shared__ int64_t s_off[kRMaxXl + 1];
  __shared__ double s_w[kRMaxXl], s_min[kRMaxXl], s_den[kRMaxXl], s_rden[kRMaxXl];
  __shared__ uint32_t s_wsum[kXlBlock / 64];
  __shared__ int s_status, s_n;
  __shared__ int64_t s_list[kXlBlock];
  // the bitonic tiles (keys, ties), or the bucket sort's kXlNB + 1 counters
  __shared__ uint64_t t_buf[2 * kXlTile + 2];
  static_assert(8 * (2 * kXlTile + 2) >= 4 * (kXlNB + 1), "counters overlay the tiles");
  uint64_t* t_key = t_buf;
  uint64_t* t_tie = t_buf + kXlTile;
  __shared__ XlScratch xs;
  const int tid = threadIdx.x;
  const XlWs w = xl_ws(ws + (int64_t)blockIdx.x * ws_each, 1 << tb, nmax, 1 << pb);
  const int64_t span = (int64_t)gridDim.x * kXlBlock;
  for (int64_t c0 = 0; c0 < p.n_queries; c0 += span) {
    if (tid == 0) s_n = 0;
    __syncthreads();
    const int64_t q = c0 + (int64_t)tid * gridDim.x + blockIdx.x;
    if (q < p.n_queries) {
      const int64_t n = p.list_off[q * p.R + p.R] - p.list_off[q * p.R];
      if (n > nmin && n <= nmax) s_list[atomicAdd(&s_n, 1)] = q;
      else if (n > nmax) p.union_count[q] = QF_QSTATUS_TOOBIG;  // beyond max_entries
    }
    __syncthreads();
    const int n = s_n;
    for (int t = 0; t < n; ++t)
      xl_one<KIND>(p, s_list[t], w, tb, pb, sort_min, s_off, s_w, s_min, s_den, s_rden,
                   s_wsum, &s_status, t_key, t_tie, &xs);
    __syncthreads();
  }
}

// ---- launch -----------------------------------------------------------------
using JoinT = JoinCfg<64, 5, 10, 6>;  // N <= 320: one wave per query (C1)
using JoinS = JoinCfg<256, 4, 11>;    // N <= 1024
using JoinM = JoinCfg<512, 10, 13, 6>;  // N <= 5120 (3 per CU with micro-unit scores)
#ifdef QF_LEARNED_512  // (A/B builds: round 5's 512-thread form)
using JoinML = JoinCfg<512, 10, 13, 4>;  // join_learned_kernel: 2 per CU (its sort's LDS)
#else
using JoinML = JoinCfg<1024, 5, 13, 8>;  // join_learned_kernel: 2 per CU, 32 waves per CU
#endif
using JoinL = JoinCfg<768, 10, 14>;   // N <= 7680
using JoinXL = JoinCfg<1024, 10, 14>; // N <= 10240 (e.g. 10 runs x top-1000; 143 KB LDS)
using SortT = SortCfg<64, 5, 8>;      // U <= 320: one wave per (query, method) (C1)
constexpr int kBsSmallUMax = 384;     // the one-wave bucket sort (C1's unions)
using SortS = SortCfg<256, 4, 4>;     // U <= 1024
using SortM = SortCfg<512, 6, 8>;     // U <= 3072
using SortL = SortCfg<768, 10, 3>;    // U <= 7680
using SortXL = SortCfg<1024, 10, 2>;  // U <= 10240

int fuse_max_entries(int wide) { return wide ? kXlNMaxWide : kXlNMax; }

template <class J>
static void launch_join(const FuseParams& p, int kind, hipStream_t st) {
  const dim3 grid = grid_for(p.n_queries), block(J::kBlock);
  if (kind == 1) hipLaunchKernelGGL((join_kernel<J, 1>), grid, block, 0, st, p);
  else hipLaunchKernelGGL((join_kernel<J, 0>), grid, block, 0, st, p);
}

template <class S>
static void launch_sort(const FuseParams& p, int umin, hipStream_t st) {
  const int M = __builtin_popcount((unsigned)p.methods);
  const int64_t groups = (p.n_queries + 7) / 8;
  hipLaunchKernelGGL((fuse_kernel<S>), grid_for(groups * 8 * M), dim3(S::kBlock), 0, st,
                     p, umin);
}

template <class S, bool FB = false>
static void launch_sort_large(const FuseParams& p, int umin, hipStream_t st, int per_cu) {
  const int64_t pairs = p.n_queries * __builtin_popcount((unsigned)p.methods);
  const int64_t cap = 256 * per_cu;  // resident workgroups (LDS / VGPR-bound)
  const int64_t grid = pairs < cap ? pairs : cap;
  hipLaunchKernelGGL((fuse_large_kernel<S, FB>), dim3((unsigned)grid), dim3(S::kBlock), 0, st,
                     p, umin);
}

// Queries above the LDS join (QF_QSTATUS_TOOBIG after it): the workspace join,
// which sorts only the unions the LDS sorts cannot hold (U > sort_min) and
// leaves the rest, unsorted with their U, to the sort kernels launched after it.
// The workspace kernel's shape for queries of up to max_entries entries: table /
// partition bits, entries per query, bytes per workgroup, and the workgroups the
// stream-ordered allocation would give it (two per CU while the workspace stays
// within 4 GB — 1.4 % of HBM; very large queries get fewer, each workgroup runs its
// queries in turn).
struct XlShape {
  int tb, pb, nmax;
  int64_t each, grid;
};
static XlShape xl_shape(int64_t n_queries, int perm32, int max_entries) {
  XlShape s{1, 0, 0, 0, 0};
  while ((1 << s.tb) < 2 * max_entries) ++s.tb;  // table load <= 1/2
  while ((1 << s.pb) < max_entries) ++s.pb;
  const int cap = perm32 ? kXlNMaxWide : kXlNMax;
  s.nmax = max_entries < cap ? max_entries : cap;
  s.each = xl_ws_bytes(1 << s.tb, s.nmax, 1 << s.pb);
  int64_t g = ((int64_t)4 << 30) / s.each;
  g = g < 1 ? 1 : (g > kXlGrid ? kXlGrid : g);
  if (n_queries < g) g = n_queries;
  s.grid = g < 1 ? 1 : g;
  return s;
}

// Whether a call takes the workspace kernel (include/qppfuse.h qf_fuse).
static bool needs_xl(int R, int max_entries) {
  return R > kRMax || max_entries > JoinXL::kNMax;
}

int64_t fuse_workspace_bytes(int64_t n_queries, int R, int max_entries, int perm32,
                             int64_t* min_bytes) {
  if (min_bytes) *min_bytes = 0;
  if (n_queries <= 0 || !needs_xl(R, max_entries)) return 0;
  const XlShape s = xl_shape(n_queries, perm32, max_entries < 1 ? 1 : max_entries);
  if (min_bytes) *min_bytes = s.each;
  return s.each * s.grid;
}

static hipError_t launch_xl(const FuseParams& p, int kind, int max_entries, int nmin,
                            int sort_min, hipStream_t st, void** ws_out, void* ws_user,
                            size_t ws_bytes) {
  const XlShape s = xl_shape(p.n_queries, p.perm32, max_entries);
  const int tb = s.tb, pb = s.pb, nmax = s.nmax;
  const int64_t each = s.each;
  int64_t g = s.grid;
  unsigned char* ws;
  if (ws_user) {  // the caller's workspace: as many workgroups as it holds (>= 1, checked)
    const int64_t fit = (int64_t)(ws_bytes / (size_t)each);
    if (fit < g) g = fit;
    if (g < 1) return hipErrorInvalidValue;
    ws = (unsigned char*)ws_user;
  } else {
    hipError_t e = hipMallocAsync(ws_out, (size_t)(each * g), st);
    if (e != hipSuccess) return e;
    ws = (unsigned char*)*ws_out;
  }
  if (kind == 1)
    hipLaunchKernelGGL((join_sort_xl_kernel<1>), dim3((unsigned)g), dim3(kXlBlock), 0, st, p,
                       nmin, ws, each, nmax, tb, pb, sort_min);
  else
    hipLaunchKernelGGL((join_sort_xl_kernel<0>), dim3((unsigned)g), dim3(kXlBlock), 0, st, p,
                       nmin, ws, each, nmax, tb, pb, sort_min);
  return hipGetLastError();
}

hipError_t fuse_launch(const FuseParams& p0, int kind, int max_entries, hipStream_t st,
                       void* ws_user, size_t ws_bytes) {
  void* ws = nullptr;
  hipError_t e = hipSuccess;
  FuseParams p = p0;
  if (p.R <= kRMax && max_entries <= JoinXL::kNMax && max_entries > JoinS::kNMax) {
    // the join kernel, then the bucket sort per (query, method) for U <= kJsUMax
    const bool learned_only = p.methods == QF_LEARNED && kind == 1 &&
                              max_entries <= JoinM::kNMax;
    if (learned_only) p.learned_reach = kLearnedUMax;
    // (Measured, not kept, round 4: every method's sort in the join's workgroup too —
    // the sums stored, each slot read back L2-hot by the thread that stored it and
    // ranked by bsort_core in the join's dead LDS: 349-352 us against join 126 +
    // bsort 202-204 us; the six sorts in turn at 3 workgroups per CU lose more than
    // the HBM re-read they save.)
    // (Measured, not kept, round 6 — profiles/r06_ab_list_join.txt: for one- and
    // two-method calls a "list-phased" join — after the insert and numbering, each
    // method's sums accumulated over u in LDS list by list (barrier-ordered, retriever
    // order, bit-identical), no contribution groups: W-CombSUM 120 vs 115 us, CombSUM
    // + RRF 154-175 vs 134 us on SURVEY 8(d)'s C2 — the groups it removes cost less
    // than its per-list passes; the method-independent cost is the hash insert and
    // the loads, which it keeps.)
    // (Measured, not kept, round 6 — profiles/r06_ab_join_sort_and_chunks.txt: the join
    // and every slot's sort in one 1,024-thread workgroup per query, each slot re-read
    // by the thread that stored it, 500-561 us against this pair's 485-503; and
    // Infinity-Cache-sized query chunks, join(chunk) then its sorts, 549-666 against
    // 499-503 — the sort is VALU / LDS-bound, so MALL-resident reads do not speed it,
    // and every chunk adds a join tail.)
    // the sorts' reach: 5,120 with the 1,024-thread configuration launched, else
    // 3,072 — a query above max_entries that the LDS join still holds (JoinM takes N <=
    // 5,120 whatever max_entries says) is then the fallback pass's (it
    // was left unsorted)
    p.fast_reach = max_entries > kJsUMax ? kFastUMaxL : kJsUMax;
    if (learned_only) {  // join + sort in one kernel (C5)
      hipLaunchKernelGGL((join_learned_kernel<JoinML>), grid_for(p.n_queries), dim3(JoinML::kBlock), 0, st,
                         p);
    } else {
      if (max_entries <= JoinM::kNMax) launch_join<JoinM>(p, kind, st);
      else if (max_entries <= JoinL::kNMax) launch_join<JoinL>(p, kind, st);
      else launch_join<JoinXL>(p, kind, st);
    }
    if (p.methods & ~QF_LEARNED) {
      const dim3 grid = grid_for((p.n_queries + 7) / 8 * 8 * __builtin_popcount((unsigned)p.methods));
      hipLaunchKernelGGL((bsort_fast_kernel<512, 0, kJsUMax, kFastBits, false, 8>), grid,
                         dim3(512), 0, st, p);
      if (max_entries > kJsUMax)  // unions above 3,072 (SURVEY §8(d)'s C2: 3,856-4,148)
        hipLaunchKernelGGL((bsort_fast_kernel<1024, kJsUMax, kFastUMaxL, kFastBitsL, true, 8>),
                           grid, dim3(1024), 0, st, p);
    }
    if ((p.methods & QF_LEARNED) && !learned_only)
      hipLaunchKernelGGL((bsort_kernel<512, 12, true>), grid_for((p.n_queries + 7) / 8 * 8),
                         dim3(512), 0, st, p);
    // unions above kJsUMax and the pairs the bucket sort marked: one pass
    launch_sort_large<SortL, true>(p, kJsUMax + 1, st, 1);
    if (max_entries > SortL::kUMax) launch_sort_large<SortXL>(p, SortL::kUMax + 1, st, 1);
    return hipGetLastError();
  }
  if (p.R > kRMax) {
    // more runs than the LDS join's masks hold: every query takes the workspace join
    e = launch_xl(p, kind, max_entries < 1 ? 1 : max_entries, -1, SortXL::kUMax, st, &ws,
                  ws_user, ws_bytes);
  } else if (max_entries <= JoinT::kNMax) {
    launch_join<JoinT>(p, kind, st);
  } else if (max_entries <= JoinS::kNMax) {
    launch_join<JoinS>(p, kind, st);
  } else {
    if (max_entries <= JoinM::kNMax) launch_join<JoinM>(p, kind, st);
    else if (max_entries <= JoinL::kNMax) launch_join<JoinL>(p, kind, st);
    else launch_join<JoinXL>(p, kind, st);
    if (max_entries > JoinXL::kNMax)
      e = launch_xl(p, kind, max_entries, JoinXL::kNMax, SortXL::kUMax, st, &ws, ws_user,
                    ws_bytes);
  }
  if (e == hipSuccess) {
    if (max_entries <= kBsSmallUMax && !(p.methods & QF_LEARNED)) {
      const int M = __builtin_popcount((unsigned)p.methods);
      hipLaunchKernelGGL((bsort_kernel<64, 9, false, kBsSmallUMax, true>),
                         grid_for((p.n_queries + 7) / 8 * 8 * M), dim3(64), 0, st, p);
    } else if (max_entries <= SortT::kUMax) {
      launch_sort<SortT>(p, 0, st);
    } else if (max_entries <= SortS::kUMax) {
      launch_sort<SortS>(p, 0, st);
    } else {
      launch_sort<SortM>(p, 0, st);
      launch_sort_large<SortL>(p, SortM::kUMax + 1, st, 1);  // the queries SortM left
      if (max_entries > SortL::kUMax) launch_sort_large<SortXL>(p, SortL::kUMax + 1, st, 1);
    }
    e = hipGetLastError();
  }
  if (ws) {
    const hipError_t f = hipFreeAsync(ws, st);
    if (e == hipSuccess) e = f;
  }
  return e;
}

// ---- fused top-k compaction (the multi-GPU gather's payload) -------------------
// out[(q*M + m)*k + i] = docid / score of rank i of method slot m of query q, for
// i < min(k, U_q); the rest of the row is padded (docid 0xFFFFFFFF, score NaN).
// One wave per (query, method) row, coalesced in i.
__global__ __launch_bounds__(256) void topk_kernel(int64_t n_queries, int32_t R,
                                                   const int64_t* __restrict__ list_off,
                                                   const int32_t* __restrict__ union_count,
                                                   const uint32_t* __restrict__ union_docid,
                                                   const void* __restrict__ perm, int perm32,
                                                   const double* __restrict__ fused,
                                                   int64_t out_stride, int32_t M, int32_t k,
                                                   uint32_t* __restrict__ out_docid,
                                                   double* __restrict__ out_score) {
  const int lane = threadIdx.x & 63;
  const int64_t row = block_id() * 4 + (threadIdx.x >> 6);  // q * M + m
  if (row >= n_queries * M) return;
  const int64_t q = row / M;
  const int m = (int)(row % M);
  const int64_t base = list_off[q * R];
  const int uc = union_count[q];
  const int n = uc < 0 ? 0 : (uc < k ? uc : k);
  const int64_t po = (int64_t)m * out_stride + base;
  const double* fz = fused + po;
  for (int i = lane; i < k; i += 64) {
    uint32_t d = 0xFFFFFFFFu;
    double sc = __longlong_as_double(0x7FF8000000000000ll);
    if (i < n) {
      const uint32_t u = perm32 ? ((const uint32_t*)perm)[po + i] : ((const uint16_t*)perm)[po + i];
      d = union_docid[base + u];
      sc = fz[u];  // scores by u, ranked through perm
    }
    out_docid[row * k + i] = d;
    out_score[row * k + i] = sc;
  }
}

hipError_t topk_launch(int64_t n_queries, int32_t R, const int64_t* list_off,
                       const int32_t* union_count, const uint32_t* union_docid,
                       const void* perm, int perm32, const double* fused, int64_t out_stride,
                       int32_t M, int32_t k, uint32_t* out_docid, double* out_score,
                       hipStream_t st) {
  const int64_t rows = n_queries * M;
  if (rows == 0 || k == 0) return hipSuccess;
  hipLaunchKernelGGL(topk_kernel, grid_for((rows + 3) / 4), dim3(256), 0, st, n_queries,
                     R, list_off, union_count, union_docid, perm, perm32, fused, out_stride, M, k,
                     out_docid, out_score);
  return hipGetLastError();
}


}  // namespace qf
