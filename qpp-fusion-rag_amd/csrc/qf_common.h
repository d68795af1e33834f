// qf_common.h — device helpers shared by the qppfuse HIP kernels (gfx950 / CDNA4).
//
// Everything here is written for a 64-lane wavefront.  The library is compiled
// with -ffp-contract=off: the reference's arithmetic is sequential IEEE double
// (Python floats, Java doubles) and an FMA contraction would change results.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

// Development stop points: QF_STOP(phase, acc, action...) marks where a development
// build (tools/dev/qf_dev_hooks.h, force-included by qppfuse._build.build_variant
// only) returns early to time the phases before it; in the library it expands to
// nothing — no branch, no computation of `acc`.
#ifndef QF_STOP
#define QF_STOP(phase, acc, ...) \
  do {                            \
  } while (0)
#endif
// Development timing probe (qf_dev_hooks.h, -DQF_CF_SCATTER): the bucket sort's scatter
// position; a probe build stores each item at its own index instead (conflict-free
// LDS addresses, wrong results) to price the scatter's bank conflicts.
#ifndef QF_DEV_SCATTER_POS
#define QF_DEV_SCATTER_POS(pos, lin) (pos)
#endif

namespace qf {

constexpr int kWave = 64;
constexpr int kBufNT = 2;  // buffer load / store cache policy: non-temporal (gfx950 "nt")
constexpr int kQppCols = 13;

// ---- wave-level primitives ------------------------------------------------

// Number of set bits of `mask` below this lane (v_mbcnt_lo/hi).
__device__ __forceinline__ uint32_t mbcnt(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

__device__ __forceinline__ uint32_t readlane_u32(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}

// Inclusive prefix sum across the 64 lanes of a wave.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}

// Same, with DPP (no LDS round trips), the GFX9 wave64 sequence: each lane adds
// the 3 lanes before it (row_shr:1,2,3 of the ORIGINAL value), then row_shr:4
// (bank_mask 0xe) and row_shr:8 (bank_mask 0xc) finish 16-lane rows, then
// row_bcast:15 (row_mask 0xa) and row_bcast:31 (row_mask 0xc) carry across rows.
// Out-of-row sources and masked lanes contribute `old` = 0.
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t v) {
  const int x0 = (int)v;
  int x = x0;
  x += __builtin_amdgcn_update_dpp(0, x0, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x0, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x0, 0x113, 0xf, 0xf, false);  // row_shr:3
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xe, false);   // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xc, false);   // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);   // row_bcast:15
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);   // row_bcast:31
  return (uint32_t)x;
}

// MIN / MAX of a u64 over the wave, result in lane 63 (DPP only: quad_perm,
// row_half_mirror and row_mirror reduce each 16-lane row, row_bcast:15/31 carry
// rows into lane 63; no ds_bpermute addresses).  Masked lanes read the identity.
#define QF_DPP_U64_STEP(x, id, ctrl, rmask, MAX)                                          \
  do {                                                                                     \
    const uint32_t _lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(id), (int)(uint32_t)(x), \
                                                               ctrl, rmask, 0xf, false);      \
    const uint32_t _hi = (uint32_t)__builtin_amdgcn_update_dpp(                            \
        (int)(id), (int)(uint32_t)((x) >> 32), ctrl, rmask, 0xf, false);                   \
    const uint64_t _o = ((uint64_t)_hi << 32) | _lo;                                       \
    x = (MAX) ? (_o > x ? _o : x) : (_o < x ? _o : x);                                     \
  } while (0)
template <bool MAX>
__device__ __forceinline__ uint64_t wave_minmax_u64_dpp(uint64_t x) {
  const uint32_t id = MAX ? 0u : 0xFFFFFFFFu;
  QF_DPP_U64_STEP(x, id, 0xB1, 0xf, MAX);   // quad_perm [1,0,3,2]
  QF_DPP_U64_STEP(x, id, 0x4E, 0xf, MAX);   // quad_perm [2,3,0,1]
  QF_DPP_U64_STEP(x, id, 0x141, 0xf, MAX);  // row_half_mirror
  QF_DPP_U64_STEP(x, id, 0x140, 0xf, MAX);  // row_mirror
  QF_DPP_U64_STEP(x, id, 0x142, 0xa, MAX);  // row_bcast:15
  QF_DPP_U64_STEP(x, id, 0x143, 0xc, MAX);  // row_bcast:31
  return x;
}
// MIN / MAX of a double over the wave, result in lane 63 (the same DPP pattern;
// fmin / fmax skip a NaN, so callers flag NaNs themselves).
#define QF_DPP_F64_STEP(x, ctrl, rmask, MAX)                                                 \
  do {                                                                                     \
    const double _id = (MAX) ? -INFINITY : INFINITY;                                       \
    const uint64_t _xb = (uint64_t)__double_as_longlong(x);                                \
    const uint64_t _ib = (uint64_t)__double_as_longlong(_id);                              \
    const uint32_t _lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)_ib,         \
                                                               (int)(uint32_t)_xb, ctrl,   \
                                                               rmask, 0xf, false);         \
    const uint32_t _hi = (uint32_t)__builtin_amdgcn_update_dpp(                            \
        (int)(uint32_t)(_ib >> 32), (int)(uint32_t)(_xb >> 32), ctrl, rmask, 0xf, false);  \
    const double _o = __longlong_as_double((long long)(((uint64_t)_hi << 32) | _lo));      \
    x = (MAX) ? fmax(x, _o) : fmin(x, _o);                                                 \
  } while (0)
template <bool MAX>
__device__ __forceinline__ double wave_minmax_f64_dpp(double x) {
  QF_DPP_F64_STEP(x, 0xB1, 0xf, MAX);
  QF_DPP_F64_STEP(x, 0x4E, 0xf, MAX);
  QF_DPP_F64_STEP(x, 0x141, 0xf, MAX);
  QF_DPP_F64_STEP(x, 0x140, 0xf, MAX);
  QF_DPP_F64_STEP(x, 0x142, 0xa, MAX);
  QF_DPP_F64_STEP(x, 0x143, 0xc, MAX);
  return x;
}
__device__ __forceinline__ double wave_min_f64_dpp(double x) { return wave_minmax_f64_dpp<false>(x); }
__device__ __forceinline__ double wave_max_f64_dpp(double x) { return wave_minmax_f64_dpp<true>(x); }

__device__ __forceinline__ uint64_t wave_min_u64_dpp(uint64_t x) {
  return wave_minmax_u64_dpp<false>(x);
}
__device__ __forceinline__ uint64_t wave_max_u64_dpp(uint64_t x) {
  return wave_minmax_u64_dpp<true>(x);
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v = fmax(v, __shfl_xor(v, d, 64));
  return v;
}
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v = fmin(v, __shfl_xor(v, d, 64));
  return v;
}
__device__ __forceinline__ uint64_t wave_or(uint64_t v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v |= __shfl_xor(v, d, 64);
  return v;
}
__device__ __forceinline__ uint64_t wave_and(uint64_t v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v &= __shfl_xor(v, d, 64);
  return v;
}

// ---- numerics ---------------------------------------------------------------

// Exact Python f"{x:.6f}" rounding, returned in micro-units: the integer m with
// m = round-half-even(x * 10^6) computed on the EXACT binary value of x (what
// CPython's correctly rounded formatting does).  fma() gives the exact sign of
// x*1e6 - c because it rounds only once.
__host__ __device__ __forceinline__ long long round6(double x) {
  double f = floor(x * 1e6);
  if (fma(x, 1e6, -f) < 0.0) f -= 1.0;
  else if (fma(x, 1e6, -(f + 1.0)) >= 0.0) f += 1.0;
  const double r = fma(x, 1e6, -(f + 0.5));
  long long m = (long long)f;
  if (r > 0.0 || (r == 0.0 && (m & 1))) m += 1;
  return m;
}

// Java's compensated summation as used by DoubleStream.sum()/average()
// (java.util.stream.Collectors.sumWithCompensation / computeFinalSum, JDK 11-17).
// QPPBridge.java calls Arrays.stream(rsvs).average() and list.stream().average().
struct Kahan {
  double s, c, simple;
};
__host__ __device__ __forceinline__ void kahan_init(Kahan& k) { k.s = 0.0; k.c = 0.0; k.simple = 0.0; }
__host__ __device__ __forceinline__ void kahan_add(Kahan& k, double v) {
  const double tmp = v - k.c;
  const double sum = k.s;
  const double velvel = sum + tmp;
  k.c = (velvel - sum) - tmp;
  k.s = velvel;
  k.simple += v;
}
// computeFinalSum in two halves, so that a serial chain can keep the first and
// leave the second to lane-parallel code: the compensated sum, then the
// fall-back to the simple sum when it is NaN and the simple sum infinite.
__host__ __device__ __forceinline__ double kahan_final_sum(const Kahan& k) {
#ifdef QF_JDK18_FINAL_SUM
  return k.s - k.c;  // JDK >= 18 (JDK-8214761)
#else
  return k.s + k.c;  // JDK 11..17
#endif
}
__host__ __device__ __forceinline__ double kahan_final_pick(double tmp, double simple) {
  return (isnan(tmp) && isinf(simple)) ? simple : tmp;
}
__host__ __device__ __forceinline__ double kahan_final(const Kahan& k) {
  return kahan_final_pick(kahan_final_sum(k), k.simple);
}

// Linear workgroup id of a grid made by grid_for() (qf_internal.h): the grid
// folds into y beyond 65,536 workgroups, x-fastest, so consecutive ids keep the
// XCD round-robin.
__device__ __forceinline__ int64_t block_id() {
  return (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
}

// ranx's min-max denominator: max(max - min, 1e-9) ("avoid division by zero",
// ranx/normalization min_max_norm, restated — ranx is not importable here: the
// rule is parity-unpinned; it only matters for ranges below 1e-9, never on
// .norm.res input whose smallest non-zero range is 1e-6).  A NaN range stays NaN
// (the callers' den > 0 test then gives the entry 0, as before).
__host__ __device__ __forceinline__ double ranx_den(double mx, double mn) {
  const double d = mx - mn;
  return d < 1e-9 ? 1e-9 : d;
}

// ---- correctly rounded quotients without a division --------------------------
// Markstein: with y = RN(1/b) and q within one ulp of a/b, the residual
// a - q*b is exact in one fma and RN(q + residual*y) = RN(a/b).  The join uses
// these in place of IEEE division sequences (~13 VALU each); tools/div_exact.hip
// checks all three against IEEE division on the GPU, bit for bit (micro_to_f64
// over every int32, recip_small over every n <= 2^24, div_small on 2^32 random
// pairs): 0 mismatches.
// m / 1e6: the double pandas parses from the "%.6f" text of m micro-units.
__device__ __forceinline__ double micro_to_f64(int32_t v) {
  const double m = (double)v;
  const double q = m * 1e-6;
  return fma(fma(-q, 1e6, m), 1e-6, q);
}
// 1 / n for 1 <= n <= 2^24: hardware reciprocal estimate and two Newton steps.
__device__ __forceinline__ double recip_small(int n) {
  const double d = (double)n;
  double r = __builtin_amdgcn_rcp(d);
  r = fma(r, fma(-d, r, 1.0), r);
  r = fma(r, fma(-d, r, 1.0), r);
  return r;
}
// w / n for 1 <= n <= 2^24 (finite w away from the subnormal range).
__device__ __forceinline__ double div_small(double w, int n) {
  const double d = (double)n, y = recip_small(n);
  const double q = w * y;
  return fma(fma(-q, d, w), y, q);
}
// a / b given y = 1 / b (IEEE, once per list) for 2^-900 <= a, b normal: the
// min-max scaling's quotient, one multiply and two fmas per element.
__device__ __forceinline__ double div_by_recip(double a, double b, double y) {
  const double q = a * y;
  return fma(fma(-q, b, a), y, q);
}
// 1 / n and w / n for any int n and double w: the division-free forms where
// they are checked exact, IEEE division elsewhere (n out of range, w zero,
// subnormal, huge, infinite or NaN — a zero w's sign is lost on the fast path).
__device__ __forceinline__ double recip_int(int n) {
  return (n >= 1 && n <= (1 << 24)) ? recip_small(n) : 1.0 / (double)n;
}
__device__ __forceinline__ double div_int(double w, int n) {
  const double aw = fabs(w);
  return (n >= 1 && n <= (1 << 24) && aw > 0x1p-900 && aw < 0x1p900) ? div_small(w, n)
                                                                     : w / (double)n;
}

// Order-preserving map of a double to uint64 (ascending), with -0.0 folded
// onto +0.0 so that the two compare equal, as Python's sort sees them.
__device__ __forceinline__ uint64_t f64_asc_key(double v) {
  if (v == 0.0) v = 0.0;
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double f64_from_asc_key(uint64_t k) {
  const uint64_t b = (k & 0x8000000000000000ull) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
  return __longlong_as_double((long long)b);
}

}  // namespace qf
