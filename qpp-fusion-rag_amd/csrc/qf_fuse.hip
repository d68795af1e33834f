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

#include "../../include/qppfuse.h"
#include "qf_common.h"
#include "qf_internal.h"

namespace qf {

constexpr int kRMax = 16;
constexpr uint32_t kEmpty = 0xFFFFFFFFu;

#ifdef QF_STAMPS
// Diagnostic build only (tools/): per-block phase cycle counts of block 0..kStampBlocks-1.
constexpr int kStampBlocks = 32768, kStampSlots = 16;
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
  uint32_t* hist;    // [256][WAVES]
  uint64_t* skey;    // [UMAX]
  uint16_t* spay;    // [UMAX]
  uint32_t* wtot;    // [WAVES] scan carries
  int* flag;         // fix-up status
  int U, rows, lane, wid, tid;
};

// One stable counting-scatter pass on an 8-bit digit digit(key).  Items are held
// in registers, wave-major: item i = (wid*rows + j)*64 + lane.  Within a wave a
// row's items are ranked by a ballot match of their digits; the row's leader
// lane claims a run of slots with one LDS atomicAdd (LDS ops of a wave execute
// in program order, so rows stay ordered without a read->write chain); the
// (digit, wave) offsets are one block-wide exclusive scan of the [digit][wave]
// counters.  Leaves the scattered sequence in skey/spay; `readback` reloads
// the registers.
template <int ITEMS, int WAVES, class Digit>
__device__ __forceinline__ void count_scatter(const SortCtx<ITEMS, WAVES>& sx,
                                              uint64_t (&key)[ITEMS], uint32_t (&pay)[ITEMS],
                                              Digit digit, bool readback) {
  static_assert(WAVES % 4 == 0 || WAVES == 1 || WAVES == 2, "4 counters per thread");
  const int lane = sx.lane, wid = sx.wid;
  int rp = sx.rows;
  asm volatile("" : "+s"(rp));
  // hist is [digit][wave]: in that flat order an exclusive scan IS the scatter
  // offset of (wave, digit) — digits ascending, waves ascending within a digit.
  uint32_t* hist = sx.hist;
  QF_STAMP_INIT();
  for (int k = lane; k < 256; k += 64) hist[k * WAVES + wid] = 0u;
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
      if (valid && before == 0) old = atomicAdd(&hist[d * WAVES + wid], (uint32_t)__popcll(peers));
      old = (uint32_t)__shfl((int)old, leader < 0 ? 0 : leader, 64);
      rank_in[j] = old + before;
    }
  }
  QF_STAMP(8);
  __syncthreads();
  QF_STAMP(9);
  // block-wide exclusive scan of the 256*WAVES counters, 4 per thread
  {
    constexpr int PER = 256 * WAVES / (64 * WAVES);  // == 4
    static_assert(PER == 4, "");
    uint4 v = *(uint4*)&hist[4 * sx.tid];
    const uint32_t t = v.x + v.y + v.z + v.w;
    const uint32_t incl = wave_incl_scan_dpp(t);
    if (lane == 63) sx.wtot[wid] = incl;
    __syncthreads();
    uint32_t pre = 0u;
#pragma unroll
    for (int w = 0; w < WAVES; ++w)
      if (w < wid) pre += sx.wtot[w];
    const uint32_t ex = pre + incl - t;
    *(uint4*)&hist[4 * sx.tid] = make_uint4(ex, ex + v.x, ex + v.x + v.y, ex + v.x + v.y + v.z);
  }
  __syncthreads();
  QF_STAMP(10);
  asm volatile("" : "+s"(rp));
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int i = (wid * rp + j) * 64 + lane;
    if (j < rp && i < sx.U) {
      const uint32_t dst = hist[digit(key[j]) * WAVES + wid] + rank_in[j];
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
//  1. LSD counting passes on the kWindow most significant bits of (key - kmin);
//  2. runs of items that agree on those 32 bits (contiguous, first-seen order,
//     almost always of length 1 or 2) are put in full-key order by a stable
//     insertion sort run by the thread at the run's start.
// A run longer than kRunMax sends the block on with LSD passes over every bit
// from bit 0: started from the order of step 1 (equal keys still first-seen)
// they give the same stable result.
constexpr int kRunMax = 48;
constexpr int kWindow = 24;  // bits sorted by LSD passes (3 passes of 8)

template <int ITEMS, int WAVES>
__device__ void sort_desc(const SortCtx<ITEMS, WAVES>& sx, uint64_t (&key)[ITEMS],
                          uint32_t (&pay)[ITEMS], uint64_t kmin, uint64_t kmax) {
  if (kmin >= kmax) return;  // all keys equal (or no items): first-seen order stands
  const int hb = 64 - __clzll((long long)(kmax - kmin));
  const int lo = hb > kWindow ? hb - kWindow : 0;
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

// Sorted items -> perm (u of rank i) and the fused score, coalesced.  Payload
// bit 15 marks a -0.0 score (the key folds -0.0 onto +0.0 so they tie, as in
// Python's sort; the value written keeps its sign, as "%.6f" prints it).
constexpr uint32_t kNegZero = 0x8000u;

template <int ITEMS, int WAVES>
__device__ __forceinline__ void write_out(const SortCtx<ITEMS, WAVES>& sx,
                                          const uint64_t (&key)[ITEMS],
                                          const uint32_t (&pay)[ITEMS], uint16_t* operm,
                                          double* ofused) {
  int ro = sx.rows;
  asm volatile("" : "+s"(ro));
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int i = (sx.wid * ro + j) * 64 + sx.lane;
    if (j < ro && i < sx.U) {
      double v = f64_from_asc_key(~key[j]);
      if (v == 0.0 && (pay[j] & kNegZero)) v = -0.0;
      operm[i] = (uint16_t)(pay[j] & ~kNegZero);
      ofused[i] = v;
    }
  }
}


// ============================================================================
// join_kernel
// ============================================================================
template <int BLOCK, int ITEMS, int TB>
struct JoinCfg {
  static constexpr int kBlock = BLOCK, kItems = ITEMS, kWaves = BLOCK / 64;
  static constexpr int kNMax = BLOCK * ITEMS, kTS = 1 << TB, kTB = TB;
  // LDS: the hash table (tkey, tmask: u32 [TS] each), later overlaid by the
  // grouped contributions gsc f64 [NMAX], gpr u32 [NMAX] and group starts u16 [NMAX]
  static constexpr int kGscOff = 0, kGprOff = 8 * kNMax, kGoOff = 12 * kNMax;
  static constexpr int kSmem = (8 * kTS > 14 * kNMax ? 8 * kTS : 14 * kNMax);
  static_assert(kTS >= kNMax, "hash table must hold every entry");
  static_assert(kNMax <= 65535, "u / group offsets are uint16");
  static_assert(kSmem <= 160 * 1024, "LDS budget");
};

template <class C, int KIND>
__global__ __launch_bounds__(C::kBlock) void join_kernel(FuseParams p) {
  constexpr int BLOCK = C::kBlock, ITEMS = C::kItems, WAVES = C::kWaves;
  constexpr int NMAX = C::kNMax, TS = C::kTS;
  __shared__ __attribute__((aligned(16))) unsigned char smem[C::kSmem];
  __shared__ int64_t s_off[kRMax + 1];
  __shared__ double s_w[kRMax], s_min[kRMax], s_den[kRMax];
  __shared__ int s_cnt[ITEMS * WAVES], s_gof[ITEMS * WAVES];
  __shared__ int s_U, s_status;
  uint32_t* tkey = (uint32_t*)smem;
  uint32_t* tmask = (uint32_t*)(smem + 4 * TS);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t q = blockIdx.x;
  if (q >= p.n_queries) return;
  const int R = p.R;
  if (tid <= R) s_off[tid] = p.list_off[q * R + tid];
  if (tid == 0) s_status = 0;
  __syncthreads();
  const int64_t base = s_off[0];
  const int64_t N64 = s_off[R] - base;
  if (N64 > NMAX) {  // uniform
    if (tid == 0) p.union_count[q] = QF_QSTATUS_TOOBIG;
    return;
  }
  const int N = (int)N64;
  if (tid < R) {
    const int64_t a = s_off[tid], b = s_off[tid + 1];
    s_w[tid] = p.weights ? p.weights[q * R + tid] : 1.0;
    // ranx min-max (norm="min-max", the fuse() default); lists are sorted
    // descending (checked below), so max / min are the end points.
    double mx = 0.0, mn = 0.0;
    if (b > a) {
      mx = ScoreIn<KIND>::load(p.score, a);
      mn = ScoreIn<KIND>::load(p.score, b - 1);
    }
    s_min[tid] = mn;
    s_den[tid] = mx - mn;
  }
  for (int i = tid * 4; i < TS; i += BLOCK * 4) {
    *(uint4*)&tkey[i] = make_uint4(kEmpty, kEmpty, kEmpty, kEmpty);
    *(uint4*)&tmask[i] = make_uint4(0u, 0u, 0u, 0u);
  }
  uint32_t dk[ITEMS];
  double sc[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {  // all loads in flight before the first use
    const int e = j * BLOCK + tid;
    dk[j] = e < N ? p.docid[base + e] : kEmpty;
    sc[j] = e < N ? ScoreIn<KIND>::load(p.score, base + e) : 0.0;
  }
  __syncthreads();
  // ---- insert: entry e = j*BLOCK + tid of list r(e) --------------------------
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
      // preconditions of the ranx methods / W-RRF (checked once, here)
      const int64_t g = base + e;
      if (g + 1 < s_off[r + 1]) {
        if ((p.methods & (QF_COMBSUM | QF_COMBMNZ | QF_RRF)) &&
            ScoreIn<KIND>::load(p.score, g + 1) > sc[j])
          status = QF_QSTATUS_UNSORTED;
        if ((p.methods & QF_WRRF) && p.rank && p.rank[g + 1] < p.rank[g])
          status = QF_QSTATUS_RANKORDER;
      }
    }
  }
  if (status) atomicMin(&s_status, status);
  __syncthreads();
  // ---- number distinct documents in first-seen order; size their groups ------
  uint32_t repm = 0u;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int e = j * BLOCK + tid;
    uint32_t pc = 0u;
    bool rep = false;
    if (e < N) {
      const uint32_t msk = tmask[dk[j]];
      rep = (uint32_t)(__ffs(msk) - 1) == rj[j];
      pc = rep ? (uint32_t)__popc(msk) : 0u;
    }
    repm |= (uint32_t)rep << j;
    const uint64_t b = ballot(rep);
    const uint32_t tot = readlane_u32(wave_incl_scan_dpp(pc), 63);
    if (lane == 0) {
      s_cnt[j * WAVES + wid] = __popcll(b);
      s_gof[j * WAVES + wid] = (int)tot;
    }
  }
  __syncthreads();
  if (wid == 0) {  // exclusive scans over the (row, wave) chunks, in entry order
    uint32_t c1 = 0, c2 = 0;
    for (int c0 = 0; c0 < ITEMS * WAVES; c0 += 64) {
      const int i = c0 + lane;
      const uint32_t v1 = i < ITEMS * WAVES ? (uint32_t)s_cnt[i] : 0u;
      const uint32_t v2 = i < ITEMS * WAVES ? (uint32_t)s_gof[i] : 0u;
      const uint32_t i1 = wave_incl_scan_dpp(v1), i2 = wave_incl_scan_dpp(v2);
      if (i < ITEMS * WAVES) {
        s_cnt[i] = (int)(c1 + i1 - v1);
        s_gof[i] = (int)(c2 + i2 - v2);
      }
      c1 += readlane_u32(i1, 63);
      c2 += readlane_u32(i2, 63);
    }
    if (lane == 0) s_U = (int)c1;
  }
  __syncthreads();
  const int U = s_U;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const bool rep = (repm >> j) & 1u;
    const uint64_t b = ballot(rep);
    uint32_t msk = 0u, pc = 0u;
    if (rep) {
      msk = tmask[dk[j]];
      pc = (uint32_t)__popc(msk);
    }
    const uint32_t gpre = wave_incl_scan_dpp(pc) - pc;
    if (rep) {
      const uint32_t u = (uint32_t)s_cnt[j * WAVES + wid] + mbcnt(b);
      const uint32_t go = (uint32_t)s_gof[j * WAVES + wid] + gpre;
      p.union_docid[base + u] = tkey[dk[j]];
      tkey[dk[j]] = u;                    // slot -> u
      tmask[dk[j]] = go | (msk << 16);    // slot -> group offset | retriever mask
    }
  }
  __syncthreads();
  // ---- every entry's place in its group (retriever order); a document's
  // first-seen entry opens the group: k == go ---------------------------------
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int e = j * BLOCK + tid;
    if (e < N) {
      const uint32_t gm = tmask[dk[j]];
      const uint32_t r = rj[j];
      const uint32_t k = (gm & 0xFFFFu) + (uint32_t)__popc((gm >> 16) & ((1u << r) - 1u));
      const uint32_t u = ((repm >> j) & 1u) ? tkey[dk[j]] : 0u;
      dk[j] = k | (u << 16);
    }
  }
  __syncthreads();  // the hash table is dead; its LDS becomes the groups
  double* gsc = (double*)(smem + C::kGscOff);
  uint32_t* gpr = (uint32_t*)(smem + C::kGprOff);
  uint16_t* ugo = (uint16_t*)(smem + C::kGoOff);
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int e = j * BLOCK + tid;
    if (e < N) {
      const uint32_t k = dk[j] & 0xFFFFu, r = rj[j];
      gsc[k] = sc[j];
      gpr[k] = (uint32_t)(base + e - s_off[r]) | (r << 16);
      if ((repm >> j) & 1u) ugo[dk[j] >> 16] = (uint16_t)k;
    }
  }
  __syncthreads();
  // ---- fused score of every document, every requested method ------------------
  const int methods = p.methods, rrf_k = p.rrf_k;
  int slot[6];
  for (int t = 0, c = 0; t < 6; ++t) {
    slot[t] = c;
    c += (methods >> t) & 1;
  }
  for (int u = tid; u < U; u += BLOCK) {
    const int gs = ugo[u], ge = u + 1 < U ? (int)ugo[u + 1] : N;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a5 = 0.0;
    for (int k = gs; k < ge; ++k) {
      const double s = gsc[k];
      const uint32_t q2 = gpr[k];
      const int r = (int)(q2 >> 16), pos = (int)(q2 & 0xFFFFu);
      if (methods & (QF_COMBSUM | QF_COMBMNZ)) {  // ranx min-max normalised score
        const double den = s_den[r];
        a0 += den > 0.0 ? (s - s_min[r]) / den : 0.0;
      }
      if (methods & QF_RRF) a1 += 1.0 / (double)(rrf_k + pos + 1);  // ranx rrf: rank = position
      if (methods & (QF_WCOMBSUM | QF_WCOMBMNZ)) a2 += s_w[r] * s;  // src/fusion.py:273
      if (methods & QF_WRRF) {                                      // src/fusion.py:374
        const int rk = p.rank ? p.rank[s_off[r] + pos] : pos + 1;
        a5 += s_w[r] / (double)(rrf_k + rk);
      }
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
  }
  if (tid == 0) p.union_count[q] = s_status ? s_status : U;
}

// ============================================================================
// fuse_kernel
// ============================================================================
template <int BLOCK, int ITEMS, int MINW>
struct SortCfg {
  static constexpr int kBlock = BLOCK, kItems = ITEMS, kWaves = BLOCK / 64, kMinWaves = MINW;
  static constexpr int kUMax = BLOCK * ITEMS;
  static constexpr int kKeyOff = 0;                                  // u64 [UMAX]
  static constexpr int kPayOff = 8 * kUMax;                          // u16 [UMAX]
  static constexpr int kHistOff = (kPayOff + 2 * kUMax + 15) & ~15;  // u32 [W][256]
  static constexpr int kSmem = kHistOff + 4 * 256 * kWaves;
  static_assert(kUMax < (int)kNegZero, "payload bit 15 is the -0.0 flag");
  static_assert(kSmem <= 160 * 1024, "LDS budget");
};

template <class C, int KIND>
__global__ __launch_bounds__(C::kBlock, C::kMinWaves) void fuse_kernel(FuseParams p, int umin) {
  constexpr int ITEMS = C::kItems, WAVES = C::kWaves, UMAX = C::kUMax;
  __shared__ __attribute__((aligned(16))) unsigned char smem[C::kSmem];
  __shared__ int s_flag;
  __shared__ uint32_t s_wtot[16];
  __shared__ unsigned long long s_kmin, s_kmax;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // block -> (query, method slot): slot-major groups of 8 queries, so that the
  // blocks resident together on an XCD (blockIdx % 8) read adjacent queries.
  const int M = __popc(p.methods);
  const int64_t grp8 = (int64_t)(blockIdx.x >> 3);
  const int64_t q = (grp8 / M) * 8 + (blockIdx.x & 7);
  const int ms = (int)(grp8 % M);
  if (q >= p.n_queries) return;
  const int U = p.union_count[q];
  if (U < 0 || U > UMAX || U < umin) return;  // error / other pass
  QF_STAMP_INIT();
  if (tid == 0) { s_kmin = ~0ull; s_kmax = 0ull; }
  __syncthreads();
  const int64_t base = p.list_off[q * p.R];
  uint64_t* skey = (uint64_t*)(smem + C::kKeyOff);
  uint16_t* spay = (uint16_t*)(smem + C::kPayOff);
  uint32_t* hist = (uint32_t*)(smem + C::kHistOff);
  SortCtx<ITEMS, WAVES> sx{hist, skey, spay, s_wtot, &s_flag, U,
                           (U + 64 * WAVES - 1) / (64 * WAVES), lane, wid, tid};
  // ---- the unsorted fused scores join_kernel left in fused[ms][u] --------------
  double* io = p.fused + (int64_t)ms * p.out_stride + base;
  uint64_t key[ITEMS];
  uint32_t pay[ITEMS];
  uint64_t kmn = ~0ull, kmx = 0ull;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int i = (wid * sx.rows + j) * 64 + lane;
    key[j] = ~0ull;
    pay[j] = (uint32_t)i;
    if (j < sx.rows && i < U) {
      const double v = io[i];
      if (v == 0.0 && __double_as_longlong(v) < 0) pay[j] |= kNegZero;
      key[j] = ~f64_asc_key(v);  // ascending sort on ~key == descending score
      kmn = min(kmn, key[j]);
      kmx = max(kmx, key[j]);
    }
  }
  block_min_max(kmn, kmx, &s_kmin, &s_kmax, lane);
  __syncthreads();
  QF_STAMP(0);
  sort_desc(sx, key, pay, (uint64_t)s_kmin, (uint64_t)s_kmax);
  QF_STAMP(1);
  write_out(sx, key, pay, p.perm + (int64_t)ms * p.out_stride + base, io);
  QF_STAMP(2);
}

// ---- launch -----------------------------------------------------------------
using JoinS = JoinCfg<256, 4, 11>;    // N <= 1024
using JoinM = JoinCfg<512, 10, 13>;   // N <= 5120
using JoinL = JoinCfg<768, 10, 14>;   // N <= 7680
using SortS = SortCfg<256, 4, 4>;     // U <= 1024
using SortM = SortCfg<512, 6, 8>;     // U <= 3072
using SortL = SortCfg<768, 10, 3>;    // U <= 7680

int fuse_max_entries() { return JoinL::kNMax; }

template <class J>
static void launch_join(const FuseParams& p, int kind, hipStream_t st) {
  dim3 grid((unsigned)p.n_queries), block(J::kBlock);
  if (kind == 1) hipLaunchKernelGGL((join_kernel<J, 1>), grid, block, 0, st, p);
  else hipLaunchKernelGGL((join_kernel<J, 0>), grid, block, 0, st, p);
}

template <class S>
static void launch_sort(const FuseParams& p, int kind, int umin, hipStream_t st) {
  const int M = __builtin_popcount((unsigned)p.methods);
  const int64_t groups = (p.n_queries + 7) / 8;
  dim3 grid((unsigned)(groups * 8 * M)), block(S::kBlock);
  if (kind == 1) hipLaunchKernelGGL((fuse_kernel<S, 1>), grid, block, 0, st, p, umin);
  else hipLaunchKernelGGL((fuse_kernel<S, 0>), grid, block, 0, st, p, umin);
}

hipError_t fuse_launch(const FuseParams& p, int kind, int max_entries, hipStream_t st) {
  if (max_entries <= JoinS::kNMax) {
    launch_join<JoinS>(p, kind, st);
    launch_sort<SortS>(p, kind, 0, st);
  } else {
    if (max_entries <= JoinM::kNMax) launch_join<JoinM>(p, kind, st);
    else launch_join<JoinL>(p, kind, st);
    launch_sort<SortM>(p, kind, 0, st);
    launch_sort<SortL>(p, kind, SortM::kUMax + 1, st);  // the queries SortM left
  }
  return hipGetLastError();
}

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

}  // namespace qf
