// qf_fuse.hip — multi-method rank fusion, one workgroup per query (gfx950).
//
// Replaces the per-row Python loops of src/fusion.py:
//   combsum / combmnz / rrf      (ranx fuse, src/fusion.py:170-230, 455-477)
//   weighted_combsum / _combmnz / weighted_rrf (src/fusion.py:237-380)
// and the per-query sort of write_runfile (src/fusion.py:480-492).
//
// Per query q (N = Σ_r |list(q,r)| entries, N <= NMAX = BLOCK*ITEMS):
//  1. Entries are loaded striped (entry e = j*BLOCK + tid), coalesced, and kept
//     in registers for the whole kernel (docid is only needed for the join).
//  2. LDS hash-join: open addressing on docid (atomicCAS), first-seen entry
//     index per slot via atomicMin.  Entry index e is retriever-major, so the
//     smallest e of a document is exactly the reference's first-seen order
//     (dict insertion order over rankers in runs order, rows in file order).
//  3. Distinct documents are compacted in first-seen order (ballot + scan):
//     u = 0..U-1, and union_docid[u] is written.
//  4. For each requested method, fused scores are accumulated in LDS in R
//     rounds, one retriever per round, separated by barriers: within a round
//     every u receives at most one contribution, so each document's sum is
//     formed in exactly the reference's order (retriever order) — bit-exact
//     IEEE double, no atomics on floats.
//  5. A stable LSD radix sort (8-bit digits, wave ballot-match ranking, one
//     LDS scatter per pass, passes over constant digits skipped) orders the
//     documents by fused score descending with ties in first-seen order —
//     Python's stable sorted(key=-score) of _ranx_to_dict / write_runfile.
//  6. perm (u of each rank) and the fused score are written, coalesced.
#include "qf_common.h"
#include "qf_internal.h"
#include "../../include/qppfuse.h"

namespace qf {

constexpr int kRMax = 16;

#ifdef QF_STAMPS
// Diagnostic build only (tools/): per-block phase cycle counts of block 0..kStampBlocks-1.
constexpr int kStampBlocks = 4096, kStampSlots = 16;
__device__ unsigned long long g_stamps[kStampBlocks * kStampSlots];
#define QF_STAMP_INIT() unsigned long long _st_prev = __builtin_amdgcn_s_memtime()
#define QF_STAMP(slot)                                                          \
  do {                                                                          \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();                 \
    if (threadIdx.x == 0 && blockIdx.x < kStampBlocks)                          \
      g_stamps[blockIdx.x * kStampSlots + (slot)] += _t - _st_prev;             \
    _st_prev = _t;                                                              \
  } while (0)
#else
#define QF_STAMP_INIT()
#define QF_STAMP(slot)
#endif
constexpr uint32_t kEmpty = 0xFFFFFFFFu;


template <int BLOCK, int ITEMS, int TB, int MINW>
struct FuseCfg {
  static constexpr int kBlock = BLOCK;
  static constexpr int kItems = ITEMS;
  static constexpr int kWaves = BLOCK / 64;
  static constexpr int kNMax = BLOCK * ITEMS;
  static constexpr int kTS = 1 << TB;
  static constexpr int kTB = TB;
  static constexpr int kMinWaves = MINW;
  // LDS: [umap u16 NMAX] then either the hash table (phase 1-2) or the
  // accumulate/sort image (phase 3), which alias.
  static constexpr int kUmapBytes = (2 * kNMax + 15) & ~15;
  static constexpr int kTableBytes = 8 * kTS;
  static constexpr int kAccOff = 0;                                // f64 / u64 [NMAX]
  static constexpr int kPayOff = kAccOff + 8 * kNMax;              // u16 [NMAX]
  static constexpr int kCntOff = kPayOff + 2 * kNMax;              // u8  [NMAX]
  static constexpr int kNegOff = (kCntOff + kNMax + 15) & ~15;     // u32 [NMAX/32]
  static constexpr int kHistOff = (kNegOff + 4 * ((kNMax + 31) / 32) + 15) & ~15;  // u32 [W][256]
  static constexpr int kPostBytes = kHistOff + 4 * 256 * kWaves;
  static constexpr int kSmem =
      kUmapBytes + (kTableBytes > kPostBytes ? kTableBytes : kPostBytes);
  static_assert(kTS >= kNMax, "hash table must hold every entry");
  static_assert(kNMax <= 65535, "perm / umap are uint16");
  static_assert(kSmem <= 160 * 1024, "LDS budget");
};

// Score as stored: int32 micro-units (exact "%.6f" text) or double.
template <int KIND>
struct ScoreIn {
  static __device__ __forceinline__ double load(const void* p, int64_t i) {
    return ((const double*)p)[i];
  }
};
template <>
struct ScoreIn<1> {
  // m / 1e6 is the nearest double to the "%.6f" text, i.e. pandas' parse.
  static __device__ __forceinline__ double load(const void* p, int64_t i) {
    return (double)((const int32_t*)p)[i] / 1e6;
  }
};


// ---- block-level helpers ------------------------------------------------------

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

template <int ITEMS, int WAVES>
struct SortCtx {
  uint32_t* hist;    // [WAVES][256]
  uint64_t* skey;    // [NMAX]
  uint16_t* spay;    // [NMAX]
  uint32_t* bstart;  // [257] bucket starts of the last counting pass
  int* flag;         // largest bucket of the last counting pass
  int U, rows, lane, wid, tid;
};

// One stable counting-scatter pass on an 8-bit digit digit(key).  Items are held
// in registers, wave-major: item i = (wid*rows + j)*64 + lane.  Within a wave a
// row's items are ranked by a ballot match of their digits; the row's leader
// lane claims a run of slots with one LDS atomicAdd (LDS ops of a wave execute
// in program order, so rows stay ordered without a read->write chain); digit
// offsets are an exclusive scan, digits ascending and waves ascending within a
// digit.  Leaves the scattered sequence in skey/spay, bucket starts in bstart
// and the largest bucket in *flag.  `readback` reloads the registers.
template <int ITEMS, int WAVES, class Digit>
__device__ __forceinline__ void count_scatter(const SortCtx<ITEMS, WAVES>& sx,
                                              uint64_t (&key)[ITEMS], uint32_t (&pay)[ITEMS],
                                              Digit digit, bool readback) {
  const int lane = sx.lane, wid = sx.wid;
  int rp = sx.rows;
  asm volatile("" : "+s"(rp));
  uint32_t* h = sx.hist + wid * 256;
  QF_STAMP_INIT();
  for (int k = lane; k < 256; k += 64) h[k] = 0u;
  uint32_t rank_in[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    rank_in[j] = 0u;
    if (j < rp) {  // wave-uniform
      const int i = (wid * rp + j) * 64 + lane;
      const bool valid = i < sx.U;
      const uint32_t d = digit(key[j]);
      uint64_t peers = ballot(valid);
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const uint64_t bb = ballot((d >> b) & 1u);
        peers &= ((d >> b) & 1u) ? bb : ~bb;
      }
      const uint32_t before = mbcnt(peers);
      const int leader = __ffsll((unsigned long long)peers) - 1;
      uint32_t old = 0u;
      if (valid && before == 0) old = atomicAdd(&h[d], (uint32_t)__popcll(peers));
      old = (uint32_t)__shfl((int)old, leader < 0 ? 0 : leader, 64);
      rank_in[j] = old + before;
    }
  }
  QF_STAMP(8);
  __syncthreads();
  QF_STAMP(9);
  if (wid == 0) {
    uint32_t run0 = 0, run1 = 0, run2 = 0, run3 = 0;
#pragma unroll
    for (int ww = 0; ww < WAVES; ++ww) {
      uint4* row = (uint4*)&sx.hist[ww * 256 + 4 * lane];
      const uint4 c = *row;
      *row = make_uint4(run0, run1, run2, run3);
      run0 += c.x; run1 += c.y; run2 += c.z; run3 += c.w;
    }
    const uint32_t tot = run0 + run1 + run2 + run3;
    const uint32_t lb = wave_incl_scan_dpp(tot) - tot;
    const uint32_t b0 = lb, b1 = lb + run0, b2 = b1 + run1, b3 = b2 + run2;
#pragma unroll
    for (int ww = 0; ww < WAVES; ++ww) {
      uint4* row = (uint4*)&sx.hist[ww * 256 + 4 * lane];
      uint4 c = *row;
      c.x += b0; c.y += b1; c.z += b2; c.w += b3;
      *row = c;
    }
    *(uint4*)&sx.bstart[4 * lane] = make_uint4(b0, b1, b2, b3);
    if (lane == 63) sx.bstart[256] = lb + tot;
    uint32_t mx = max(max(run0, run1), max(run2, run3));
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, d, 64));
    if (lane == 0) *sx.flag = (int)mx;
  }
  __syncthreads();
  QF_STAMP(10);
  asm volatile("" : "+s"(rp));
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int i = (wid * rp + j) * 64 + lane;
    if (j < rp && i < sx.U) {
      const uint32_t dst = h[digit(key[j])] + rank_in[j];
      sx.skey[dst] = key[j];
      sx.spay[dst] = (uint16_t)pay[j];
    }
  }
  QF_STAMP(11);
  __syncthreads();
  QF_STAMP(12);
  if (readback) {
    asm volatile("" : "+s"(rp));
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const int i = (wid * rp + j) * 64 + lane;
      if (j < rp && i < sx.U) {
        key[j] = sx.skey[i];
        pay[j] = sx.spay[i];
      }
    }
  }
  QF_STAMP(13);
}

// digit(k) = ((k - kmin) >> sh) & 0xFF.
struct Digit {
  uint64_t base;
  int sh;
  __device__ __forceinline__ uint32_t operator()(uint64_t k) const {
    return (uint32_t)((k - base) >> sh) & 0xFFu;
  }
};

// Stable sort of the items by key ascending (keys are ~orderable(score): scores
// descending; ties keep input = first-seen order).  kmin / kmax: extreme keys.
//  1. LSD counting passes on the 32 most significant bits of (key - kmin);
//  2. runs of items that agree on those 32 bits (contiguous, first-seen order,
//     almost always of length 1 or 2) are put in full-key order by a stable
//     insertion sort run by the thread at the run's start.
// A run longer than kRunMax sends the block on with LSD passes over every bit
// from bit 0: started from the order of step 1 (equal keys still first-seen)
// they give the same stable result.
constexpr int kRunMax = 64;

template <int ITEMS, int WAVES>
__device__ void sort_desc(const SortCtx<ITEMS, WAVES>& sx, uint64_t (&key)[ITEMS],
                          uint32_t (&pay)[ITEMS], uint64_t kmin, uint64_t kmax) {
  if (kmin >= kmax) return;  // all keys equal (or no items): first-seen order stands
  const int hb = 64 - __clzll((long long)(kmax - kmin));
  const int lo = hb > 32 ? hb - 32 : 0;
  int sh = lo;
  bool fallback = false;
#pragma unroll 1
  while (true) {
    count_scatter(sx, key, pay, Digit{kmin, sh}, true);
    sh += 8;
    if (sh < hb) continue;
    if (fallback || lo == 0) return;
    // -- fix up runs that agree on the window ------------------------------------
    // count_scatter left the sorted sequence in skey/spay.
    if (sx.tid == 0) *sx.flag = 0;
    __syncthreads();
    bool moved = false;
    for (int i = sx.tid; i < sx.U; i += WAVES * 64) {
      const uint64_t hk = (sx.skey[i] - kmin) >> lo;
      if (i > 0 && ((sx.skey[i - 1] - kmin) >> lo) == hk) continue;  // not a run start
      if (i + 1 >= sx.U || ((sx.skey[i + 1] - kmin) >> lo) != hk) continue;  // length 1
      int L = 2;
      while (i + L < sx.U && ((sx.skey[i + L] - kmin) >> lo) == hk && L <= kRunMax) ++L;
      if (L > kRunMax) { atomicOr(sx.flag, 1); continue; }
      for (int a = i + 1; a < i + L; ++a) {  // stable insertion sort on the full key
        const uint64_t k = sx.skey[a];
        const uint16_t v = sx.spay[a];
        int b = a - 1;
        while (b >= i && sx.skey[b] > k) {
          sx.skey[b + 1] = sx.skey[b];
          sx.spay[b + 1] = sx.spay[b];
          --b;
        }
        if (b + 1 != a) {
          sx.skey[b + 1] = k;
          sx.spay[b + 1] = v;
          moved = true;
        }
      }
    }
    if (moved) atomicOr(sx.flag, 2);
    __syncthreads();
    const int f = *sx.flag;  // block-uniform
    if (f & 1) {             // a run too long: finish with full LSD passes
      fallback = true;
      sh = 0;
      continue;              // registers still hold the step-1 order
    }
    if (f & 2) {
      int rp = sx.rows;
      asm volatile("" : "+s"(rp));
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        const int i = (sx.wid * rp + j) * 64 + sx.lane;
        if (j < rp && i < sx.U) {
          key[j] = sx.skey[i];
          pay[j] = sx.spay[i];
        }
      }
    }
    return;
  }
}

// Sorted items -> perm (u of rank i) and the fused score, coalesced.
template <int ITEMS, int WAVES>
__device__ __forceinline__ void write_out(const SortCtx<ITEMS, WAVES>& sx,
                                          const uint64_t (&key)[ITEMS],
                                          const uint32_t (&pay)[ITEMS], const uint32_t* negz,
                                          uint16_t* operm, double* ofused) {
  int ro = sx.rows;
  asm volatile("" : "+s"(ro));
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int i = (sx.wid * ro + j) * 64 + sx.lane;
    if (j < ro && i < sx.U) {
      double v = f64_from_asc_key(~key[j]);
      if (v == 0.0 && ((negz[pay[j] >> 5] >> (pay[j] & 31)) & 1u)) v = -0.0;
      operm[i] = (uint16_t)pay[j];
      ofused[i] = v;
    }
  }
}

template <class C, int KIND>
__global__ __launch_bounds__(C::kBlock, C::kMinWaves) void fuse_kernel(FuseParams p) {
  constexpr int BLOCK = C::kBlock, ITEMS = C::kItems, WAVES = C::kWaves;
  constexpr int NMAX = C::kNMax, TS = C::kTS;
  __shared__ __attribute__((aligned(16))) unsigned char smem[C::kSmem];
  __shared__ int64_t s_off[kRMax + 1];
  __shared__ double s_w[kRMax], s_min[kRMax], s_den[kRMax];
  __shared__ int s_chunk[ITEMS * WAVES];
  __shared__ int s_U, s_status, s_flag;
  __shared__ __attribute__((aligned(16))) uint32_t s_bstart[260];
  __shared__ unsigned long long s_or[2], s_and[2];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t q = blockIdx.x;
  if (q >= p.n_queries) return;
  const int R = p.R;
  QF_STAMP_INIT();

  if (tid <= R) s_off[tid] = p.list_off[q * R + tid];
  if (tid == 0) s_status = 0;
  __syncthreads();
  const int64_t base = s_off[0];
  const int64_t N64 = s_off[R] - base;
  if (N64 > NMAX) {  // uniform: every thread sees the same offsets
    if (tid == 0) p.union_count[q] = QF_QSTATUS_TOOBIG;
    return;
  }
  const int N = (int)N64;
  if (tid < R) {
    const int64_t a = s_off[tid], b = s_off[tid + 1];
    s_w[tid] = p.weights ? p.weights[q * R + tid] : 1.0;
    // ranx min-max (norm="min-max", the fuse() default).  Lists are sorted
    // descending (checked below), so max / min are the end points.
    double mx = 0.0, mn = 0.0;
    if (b > a) {
      mx = ScoreIn<KIND>::load(p.score, a);
      mn = ScoreIn<KIND>::load(p.score, b - 1);
    }
    s_min[tid] = mn;
    s_den[tid] = mx - mn;
  }

  uint16_t* umap = (uint16_t*)smem;                      // entry e -> u
  unsigned char* img = smem + C::kUmapBytes;
  // ---- phase 1: LDS hash insert -------------------------------------------
  uint32_t* tkey = (uint32_t*)img;
  uint32_t* tmask = tkey + TS;  // retrievers holding the slot's docid; later slot -> u
  for (int i = tid * 4; i < TS; i += BLOCK * 4) {
    *(uint4*)&tkey[i] = make_uint4(kEmpty, kEmpty, kEmpty, kEmpty);
    *(uint4*)&tmask[i] = make_uint4(0u, 0u, 0u, 0u);
  }
  uint32_t dk[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {  // all loads in flight before the first use
    const int e = j * BLOCK + tid;
    dk[j] = e < N ? p.docid[base + e] : kEmpty;
  }
  __syncthreads();
  // Entry e = j*BLOCK + tid belongs to list r(e); lists are retriever-major, so
  // a document's first-seen entry is its entry in the lowest retriever holding
  // it: the lowest bit of the slot's retriever mask.  A bit already set when an
  // entry ORs it in means the docid repeats inside one list (unsupported).
  int status = 0;
  uint32_t rj[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int e = j * BLOCK + tid;
    rj[j] = 0u;
    if (e < N) {
      const uint32_t d = dk[j];
      if (d == kEmpty) status = QF_QSTATUS_BADDOC;
      int r = 0;
      while (base + e >= s_off[r + 1]) ++r;
      rj[j] = (uint32_t)r;
      uint32_t h = (d * 0x9E3779B1u) >> (32 - C::kTB);
      while (true) {
        const uint32_t prev = atomicCAS(&tkey[h], kEmpty, d);
        if (prev == kEmpty || prev == d) break;
        h = (h + 1) & (TS - 1);
      }
      const uint32_t old = atomicOr(&tmask[h], 1u << r);
      if ((old >> r) & 1u) status = QF_QSTATUS_DUPDOC;
      dk[j] = h;  // keep the slot
    }
  }
  if (status) atomicMin(&s_status, status);
  __syncthreads();
  QF_STAMP(0);

  // ---- phase 2: distinct documents in first-seen order --------------------
  uint32_t repm = 0u;  // bit j: entry j is its document's first occurrence
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int e = j * BLOCK + tid;
    const bool rep = (e < N) && (uint32_t)(__ffs(tmask[dk[j]]) - 1) == rj[j];
    repm |= (uint32_t)rep << j;
    const uint64_t b = ballot(rep);
    if (lane == 0) s_chunk[j * WAVES + wid] = __popcll(b);
  }
  __syncthreads();
  if (wid == 0) {
    uint32_t carry = 0;
    for (int c0 = 0; c0 < ITEMS * WAVES; c0 += 64) {
      const int i = c0 + lane;
      const uint32_t v = i < ITEMS * WAVES ? (uint32_t)s_chunk[i] : 0u;
      const uint32_t incl = wave_incl_scan(v);
      if (i < ITEMS * WAVES) s_chunk[i] = (int)(carry + incl - v);
      carry += __shfl(incl, 63, 64);
    }
    if (lane == 0) s_U = (int)carry;
  }
  __syncthreads();
  const int U = s_U;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const bool rep = (repm >> j) & 1u;
    const uint64_t b = ballot(rep);
    if (rep) {
      const uint32_t u = (uint32_t)s_chunk[j * WAVES + wid] + mbcnt(b);
      p.union_docid[base + u] = tkey[dk[j]];
      tmask[dk[j]] = u;  // slot -> u (only the representative writes)
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int e = j * BLOCK + tid;
    if (e < N) umap[e] = (uint16_t)tmask[dk[j]];
  }
  __syncthreads();  // hash table dead from here; its LDS is re-used below
  QF_STAMP(1);

  double* acc = (double*)(img + C::kAccOff);
  uint64_t* skey = (uint64_t*)(img + C::kAccOff);
  uint16_t* spay = (uint16_t*)(img + C::kPayOff);
  uint8_t* cnt = (uint8_t*)(img + C::kCntOff);
  uint32_t* negz = (uint32_t*)(img + C::kNegOff);
  uint32_t* hist = (uint32_t*)(img + C::kHistOff);
  SortCtx<ITEMS, WAVES> sx{hist, skey, spay, s_bstart, &s_flag, U,
                           (U + 64 * WAVES - 1) / (64 * WAVES), lane, wid, tid};

  // One job per method, in method-bit order.  CombMNZ / W-CombMNZ are the SUM
  // family's sums times the per-document count (ranx comb_mnz, src/fusion.py:327):
  // right after their SUM job they reuse its sorted sums (no accumulation rounds).
  uint64_t key[ITEMS];
  uint32_t pay[ITEMS];
  bool first_family = true;
  bool have_sorted_sum = false;
#pragma unroll 1
  for (int job = 0; job < 6; ++job) {
    if (!((p.methods >> job) & 1)) { have_sorted_sum = false; continue; }
    const bool is_mnz = job == 1 || job == 4;
    const int fam = is_mnz ? job - 1 : job;  // 0 sum, 2 rrf, 3 wsum, 5 wrrf
    if (tid == 0) { s_or[0] = ~0ull; s_and[0] = 0ull; }  // min / max key
    if (!(is_mnz && have_sorted_sum)) {
      // -- zero accumulators ----------------------------------------------------
      for (int i = tid; i < U; i += BLOCK) acc[i] = 0.0;
      if (first_family)
        for (int i = tid; i < U; i += BLOCK) cnt[i] = 0;
      for (int i = tid; i < (NMAX + 31) / 32; i += BLOCK) negz[i] = 0u;
      __syncthreads();
      QF_STAMP(2);
      // -- ordered accumulation: one retriever (list) per round -----------------
      // Scores for round r+1 are loaded before round r's barrier.
      const bool need_score = fam == 0 || fam == 3;
      int status2 = 0;
      constexpr int PF = 2;  // entries per thread prefetched per round (K <= 2*BLOCK)
      double nxt[PF];
      auto fetch = [&](int r, double (&dst)[PF]) {
        const int e0 = (int)(s_off[r] - base), e1 = (int)(s_off[r + 1] - base);
#pragma unroll
        for (int t = 0; t < PF; ++t) {
          const int e = e0 + tid + t * BLOCK;
          dst[t] = (need_score && e < e1) ? ScoreIn<KIND>::load(p.score, base + e) : 0.0;
        }
      };
      fetch(0, nxt);
#pragma unroll 1
      for (int r = 0; r < R; ++r) {
        double cur[PF];
#pragma unroll
        for (int t = 0; t < PF; ++t) cur[t] = nxt[t];
        if (r + 1 < R) fetch(r + 1, nxt);
        const double w = s_w[r], mn = s_min[r], den = s_den[r];
        const int e0 = (int)(s_off[r] - base), e1 = (int)(s_off[r + 1] - base);
        for (int e = e0 + tid, t = 0; e < e1; e += BLOCK, ++t) {
          const int pos = e - e0;
          double sj = 0.0;
          if (need_score) {
            if (t < PF) {
#pragma unroll
              for (int tt = 0; tt < PF; ++tt)
                if (tt == t) sj = cur[tt];
            } else {
              sj = ScoreIn<KIND>::load(p.score, base + e);
            }
          }
          double c;
          if (fam == 0) c = den > 0.0 ? (sj - mn) / den : 0.0;          // ranx min-max
          else if (fam == 2) c = 1.0 / (double)(p.rrf_k + pos + 1);     // ranx rrf
          else if (fam == 3) c = w * sj;                                // fusion.py:273
          else c = w / (double)(p.rrf_k + (p.rank ? p.rank[base + e] : pos + 1));  // :374
          const uint32_t u = umap[e];
          acc[u] += c;
          if (first_family) {
            cnt[u] += 1;
            // preconditions: scores non-increasing in a list when a ranx method
            // (min-max end points, RRF rank = position) is requested; rank column
            // non-decreasing when W-RRF reads it (first-seen = rank order).
            if (e + 1 < e1) {
              if ((p.methods & (QF_COMBSUM | QF_COMBMNZ | QF_RRF)) &&
                  ScoreIn<KIND>::load(p.score, base + e + 1) >
                      ScoreIn<KIND>::load(p.score, base + e))
                status2 = QF_QSTATUS_UNSORTED;
              if ((p.methods & QF_WRRF) && p.rank && p.rank[base + e + 1] < p.rank[base + e])
                status2 = QF_QSTATUS_RANKORDER;
            }
          }
        }
        __syncthreads();
      }
      if (first_family) {
        if (status2) atomicMin(&s_status, status2);
        __syncthreads();
        if (tid == 0) p.union_count[q] = s_status ? s_status : U;
      }
      first_family = false;
      QF_STAMP(3);
      // -- keys in first-seen order -----------------------------------------------
      int rowsk = sx.rows;
      asm volatile("" : "+s"(rowsk));  // keep per-item addresses out of loop-invariant code
      uint64_t kmn = ~0ull, kmx = 0ull;
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        const int i = (wid * rowsk + j) * 64 + lane;
        key[j] = ~0ull;
        pay[j] = (uint32_t)i;
        if (j < rowsk && i < U) {
          double v = acc[i];
          if (is_mnz) v = v * (double)cnt[i];
          if (v == 0.0 && __double_as_longlong(v) < 0) atomicOr(&negz[i >> 5], 1u << (i & 31));
          key[j] = ~f64_asc_key(v);  // ascending sort on ~key == descending score
          kmn = min(kmn, key[j]);
          kmx = max(kmx, key[j]);
        }
      }
      block_min_max(kmn, kmx, &s_or[0], &s_and[0], lane);
      __syncthreads();  // acc no longer read; skey may be written
    } else {
      // -- MNZ from the sorted SUM items, scattered back to first-seen (u) order
      //    so that the stable sort breaks ties by first-seen order again.
      uint64_t kmn = ~0ull, kmx = 0ull;
      int rp = sx.rows;
      asm volatile("" : "+s"(rp));
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        const int i = (wid * rp + j) * 64 + lane;
        if (j < rp && i < U) {
          double v = f64_from_asc_key(~key[j]);
          if (v == 0.0 && ((negz[pay[j] >> 5] >> (pay[j] & 31)) & 1u)) v = -0.0;
          v = v * (double)cnt[pay[j]];
          const uint64_t k2 = ~f64_asc_key(v);
          skey[pay[j]] = k2;
          kmn = min(kmn, k2);
          kmx = max(kmx, k2);
        }
      }
      block_min_max(kmn, kmx, &s_or[0], &s_and[0], lane);
      __syncthreads();
      asm volatile("" : "+s"(rp));
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        const int i = (wid * rp + j) * 64 + lane;
        pay[j] = (uint32_t)i;
        key[j] = (j < rp && i < U) ? skey[i] : ~0ull;
      }
      __syncthreads();
    }
    QF_STAMP(4);
    sort_desc(sx, key, pay, (uint64_t)s_or[0], (uint64_t)s_and[0]);
    QF_STAMP(5);
    const int slot = __popc(p.methods & ((1 << job) - 1));
    write_out(sx, key, pay, negz, p.perm + (int64_t)slot * p.out_stride + base,
              p.fused + (int64_t)slot * p.out_stride + base);
    have_sorted_sum = !is_mnz && (fam == 0 || fam == 3);
    __syncthreads();  // skey / negz / acc are rewritten by the next job
    QF_STAMP(6);
  }
}

// ---- launch -----------------------------------------------------------------
using CfgS = FuseCfg<256, 4, 11, 4>;    // N <= 1024   (e.g. 3 x top-100)
using CfgM = FuseCfg<512, 10, 13, 4>;   // N <= 5120   (5 x top-1000)
using CfgL = FuseCfg<768, 10, 13, 3>;   // N <= 7680   (7 x top-1000)

template <class C>
static hipError_t launch_cfg(const FuseParams& p, int kind, hipStream_t st) {
  dim3 grid((unsigned)p.n_queries), block(C::kBlock);
  if (kind == 1) hipLaunchKernelGGL((fuse_kernel<C, 1>), grid, block, 0, st, p);
  else hipLaunchKernelGGL((fuse_kernel<C, 0>), grid, block, 0, st, p);
  return hipGetLastError();
}

int fuse_max_entries() { return CfgL::kNMax; }

#ifdef QF_STAMPS
extern "C" int qf_debug_stamps(unsigned long long* host, int n, int clear) {
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * n) != hipSuccess)
    return 1;
  if (clear) {
    static unsigned long long zeros[kStampBlocks * kStampSlots];
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), zeros, sizeof zeros) != hipSuccess) return 1;
  }
  return 0;
}
#endif

hipError_t fuse_launch(const FuseParams& p, int kind, int max_entries, hipStream_t st) {
  if (max_entries <= CfgS::kNMax) return launch_cfg<CfgS>(p, kind, st);
  if (max_entries <= CfgM::kNMax) return launch_cfg<CfgM>(p, kind, st);
  return launch_cfg<CfgL>(p, kind, st);
}

}  // namespace qf
