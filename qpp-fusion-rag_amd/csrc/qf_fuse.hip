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

template <class C, int KIND>
__global__ __launch_bounds__(C::kBlock, C::kMinWaves) void fuse_kernel(FuseParams p) {
  constexpr int BLOCK = C::kBlock, ITEMS = C::kItems, WAVES = C::kWaves;
  constexpr int NMAX = C::kNMax, TS = C::kTS;
  __shared__ __attribute__((aligned(16))) unsigned char smem[C::kSmem];
  __shared__ int64_t s_off[kRMax + 1];
  __shared__ double s_w[kRMax], s_min[kRMax], s_den[kRMax];
  __shared__ int s_chunk[ITEMS * WAVES];
  __shared__ int s_U, s_status;
  __shared__ unsigned long long s_or, s_and;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t q = blockIdx.x;
  if (q >= p.n_queries) return;
  const int R = p.R;

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

  double* acc = (double*)(img + C::kAccOff);
  uint64_t* skey = (uint64_t*)(img + C::kAccOff);
  uint16_t* spay = (uint16_t*)(img + C::kPayOff);
  uint8_t* cnt = (uint8_t*)(img + C::kCntOff);
  uint32_t* negz = (uint32_t*)(img + C::kNegOff);
  uint32_t* hist = (uint32_t*)(img + C::kHistOff);
  // Sort layout: rows of 64 items per wave, wave-major (item i = wid*64*rows +
  // j*64 + lane): every wave holds the same number of rows.
  const int rows = (U + 64 * WAVES - 1) / (64 * WAVES);

  int slot_out = 0;
  bool first_method = true;
#pragma unroll 1
  for (int m = 0; m < 6; ++m) {
    if (!((p.methods >> m) & 1)) continue;
    // -- zero accumulators ----------------------------------------------------
    for (int i = tid; i < U; i += BLOCK) acc[i] = 0.0;
    if (first_method)
      for (int i = tid; i < U; i += BLOCK) cnt[i] = 0;
    for (int i = tid; i < (NMAX + 31) / 32; i += BLOCK) negz[i] = 0u;
    if (tid == 0) { s_or = 0ull; s_and = ~0ull; }
    __syncthreads();
    // -- ordered accumulation: one retriever (list) per round -----------------
    int status2 = 0;
#pragma unroll 1
    for (int r = 0; r < R; ++r) {
      const double w = s_w[r], mn = s_min[r], den = s_den[r];
      const int e0 = (int)(s_off[r] - base), e1 = (int)(s_off[r + 1] - base);
      for (int e = e0 + tid; e < e1; e += BLOCK) {
        const int pos = e - e0;
        double c;
        switch (m) {
          case 0:
          case 1: {  // ranx min-max normalised score
            const double sj = ScoreIn<KIND>::load(p.score, base + e);
            c = den > 0.0 ? (sj - mn) / den : 0.0;
          } break;
          case 2: c = 1.0 / (double)(p.rrf_k + pos + 1); break;  // ranx rrf
          case 3:
          case 4: c = w * ScoreIn<KIND>::load(p.score, base + e); break;  // fusion.py:273
          default: {                                                     // fusion.py:374
            const int rk = p.rank ? p.rank[base + e] : pos + 1;
            c = w / (double)(p.rrf_k + rk);
          }
        }
        const uint32_t u = umap[e];
        acc[u] += c;
        if (first_method) {
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
    if (first_method) {
      if (status2) atomicMin(&s_status, status2);
      __syncthreads();
      if (tid == 0) p.union_count[q] = s_status ? s_status : U;
    }
    first_method = false;
    // -- keys -----------------------------------------------------------------
    // `rows` is re-materialised opaquely in each phase: otherwise the compiler
    // hoists every item's LDS addresses out of the loops and keeps them live.
    int rowsk = rows;
    asm volatile("" : "+s"(rowsk));
    uint64_t key[ITEMS];
    uint32_t pay[ITEMS];
    uint64_t kor = 0ull, kand = ~0ull;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const int i = (wid * rowsk + j) * 64 + lane;
      key[j] = ~0ull;
      pay[j] = (uint32_t)i;
      if (j < rowsk && i < U) {
        double v = acc[i];
        if (m == 1 || m == 4) v = v * (double)cnt[i];  // CombMNZ: sum x count
        if (v == 0.0 && __double_as_longlong(v) < 0) atomicOr(&negz[i >> 5], 1u << (i & 31));
        key[j] = ~f64_asc_key(v);  // ascending radix on ~key == descending score
        kor |= key[j];
        kand &= key[j];
      }
    }
    kor = wave_or(kor);
    kand = wave_and(kand);
    if (lane == 0) {
      atomicOr(&s_or, (unsigned long long)kor);
      atomicAnd(&s_and, (unsigned long long)kand);
    }
    __syncthreads();  // acc no longer read; skey may be written
    const uint64_t varying = (uint64_t)(s_or ^ s_and);

    // -- stable LSD radix sort, 8-bit digits -------------------------------------
#pragma unroll 1
    for (int sh = 0; sh < 64; sh += 8) {
      if (((varying >> sh) & 0xFFull) == 0ull) continue;  // block-uniform
      int rp = rows;
      asm volatile("" : "+s"(rp));
      uint32_t* h = hist + wid * 256;
      for (int k = lane; k < 256; k += 64) h[k] = 0u;
      uint32_t rank_in[ITEMS];
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        rank_in[j] = 0u;
        if (j < rp) {  // wave-uniform
          const int i = (wid * rp + j) * 64 + lane;
          const bool valid = i < U;
          const uint32_t d = (uint32_t)(key[j] >> sh) & 0xFFu;
          uint64_t peers = ballot(valid);
#pragma unroll
          for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = ballot(bit);
            peers &= bit ? bb : ~bb;
          }
          if (valid) {
            const uint32_t before = mbcnt(peers);
            const uint32_t c0 = h[d];
            rank_in[j] = c0 + before;
            if (before == 0) h[d] = c0 + (uint32_t)__popcll(peers);
          }
        }
        __builtin_amdgcn_sched_barrier(0);  // one row at a time: bounds live ranges
      }
      __syncthreads();
      if (wid == 0) {  // digit offsets: digits ascending, waves ascending within a digit
        uint32_t run0 = 0, run1 = 0, run2 = 0, run3 = 0;
        for (int ww = 0; ww < WAVES; ++ww) {
          uint4* row = (uint4*)&hist[ww * 256 + 4 * lane];
          const uint4 c = *row;
          *row = make_uint4(run0, run1, run2, run3);
          run0 += c.x; run1 += c.y; run2 += c.z; run3 += c.w;
        }
        const uint32_t tot = run0 + run1 + run2 + run3;
        const uint32_t lb = wave_incl_scan(tot) - tot;
        const uint32_t b0 = lb, b1 = lb + run0, b2 = b1 + run1, b3 = b2 + run2;
        for (int ww = 0; ww < WAVES; ++ww) {
          uint4* row = (uint4*)&hist[ww * 256 + 4 * lane];
          uint4 c = *row;
          c.x += b0; c.y += b1; c.z += b2; c.w += b3;
          *row = c;
        }
      }
      __syncthreads();
      asm volatile("" : "+s"(rp));
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        const int i = (wid * rp + j) * 64 + lane;
        if (j < rp && i < U) {
          const uint32_t d = (uint32_t)(key[j] >> sh) & 0xFFu;
          const uint32_t dst = h[d] + rank_in[j];
          skey[dst] = key[j];
          spay[dst] = (uint16_t)pay[j];
        }
      }
      __syncthreads();
      asm volatile("" : "+s"(rp));
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        const int i = (wid * rp + j) * 64 + lane;
        if (j < rp && i < U) {
          key[j] = skey[i];
          pay[j] = spay[i];
        }
      }
    }
    // -- write sorted output -----------------------------------------------------
    uint16_t* operm = p.perm + (int64_t)slot_out * p.out_stride + base;
    double* ofused = p.fused + (int64_t)slot_out * p.out_stride + base;
    int ro = rows;
    asm volatile("" : "+s"(ro));
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const int i = (wid * ro + j) * 64 + lane;
      if (j < ro && i < U) {
        double v = f64_from_asc_key(~key[j]);
        if (v == 0.0 && ((negz[pay[j] >> 5] >> (pay[j] & 31)) & 1u)) v = -0.0;
        operm[i] = (uint16_t)pay[j];
        ofused[i] = v;
      }
    }
    ++slot_out;
    __syncthreads();  // skey / negz are rewritten by the next method
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

hipError_t fuse_launch(const FuseParams& p, int kind, int max_entries, hipStream_t st) {
  if (max_entries <= CfgS::kNMax) return launch_cfg<CfgS>(p, kind, st);
  if (max_entries <= CfgM::kNMax) return launch_cfg<CfgM>(p, kind, st);
  return launch_cfg<CfgL>(p, kind, st);
}

}  // namespace qf
