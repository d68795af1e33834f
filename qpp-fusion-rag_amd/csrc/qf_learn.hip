// qf_learn.hip — learned-fusion weights on gfx950: LightGBM inference + the
// reference's weight normalisation.
//
// Replaces learned_fusion's model step (src/fusion.py:407-434):
//   X[q, j*n_qpp + c] = qpp[q][retriever j][c]            (built by the caller)
//   pred = model.predict(X)   MultiOutputLGBM / PerRetrieverLGBM: one LightGBM
//                             booster per retriever (src/models/
//                             lightgbm_models.py:114-123, 232-241)
//   _normalize_weights: clip(pred, 0, None); s = pred.sum(axis=1); s[s == 0] = 1;
//                       pred / s                          (src/models/base.py:120-125)
//   weight of run r = pred[q][model index of r], or 1/n_retrievers for a run the
//   model does not know (src/fusion.py:440)
//
// gbdt_predict_kernel — one wave per row: the lanes walk the model's trees
//   (LightGBM NumericalDecision; see qppfuse/lgbm.py), then each booster's leaf
//   values are added in tree order from 0.0, as GBDT::PredictRaw does.  The
//   model (≈4.5 k nodes for the reference's NQ model) stays in L1/L2.
// learned_weights_kernel — one thread per query: numpy's clip (NaN kept, -0.0
//   becomes +0.0 — measured on numpy 2.2), numpy's row sum (0.0 + pairwise_sum: sequential below 8
//   values, 8 accumulators from 8), the zero guard and the division.
// mlp_weights_kernel — FusionMLP.predict (src/models/mlp_model.py:254-274), one
//   wave per query: the selected QPP columns (_filter_features, :104-122) rounded
//   to float32 (torch.FloatTensor), Linear -> ReLU -> (Dropout: identity in eval)
//   ... -> Linear, softmax, then _normalize_weights in float32.  The order of every
//   float32 operation is fixed (no contraction: each product and sum rounds):
//     y[o] = (sum_i x[i] * W[o][i], i ascending, from +0.0) + b[o]
//     softmax: m = max z; e = float(exp(double(z - m))); s = sum e (ascending,
//              from 0); p = e / s
//   so oracle/mlp_oracle.py restates it bit for bit.  torch's CPU GEMM / softmax
//   (and the MPS device the reference trained on) accumulate in other orders:
//   tests/test_gpu_learned.py holds the two within float32 rounding.
#include <math.h>

#include "../../include/qppfuse.h"
#include "qf_common.h"
#include "qf_internal.h"
#include "qf_lists.h"

namespace qf {

// numpy's pairwise_sum for n < 128 (numpy/_core/src/umath/loops_utils.h.src)
__device__ __forceinline__ double np_pairwise_sum(const double* a, int n) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  double r[8];
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}

// One wave per row: the lanes walk the model's trees in parallel (tree c0 + lane
// of each 64-tree chunk, the row's features staged in LDS), then lane b adds
// booster b's leaf values of the chunk in tree order onto its running sum — the
// serial GBDT::PredictRaw sum from 0.0, tree by tree, bit for bit.  (Was: one
// thread per (row, booster) walking its ~30 trees serially — C5: 17,260 threads,
// ~270 waves on 256 CUs, each a chain of ~30 tree walks of dependent loads.)
// Round 4: the whole model is staged in LDS when it fits (the reference's NQ
// model: 4,470 nodes + 4,619 leaves = 133 KB with the rows), one 16-wave
// workgroup per CU, so a tree level costs two dependent LDS reads instead of a
// dependent L1 / L2 load; a larger model walks the global arrays (same code).
constexpr int kGbdtWaves = 16;
constexpr int kGbdtMaxFeatures = 256;      // staged in LDS; more features: read from X
constexpr int kGbdtLds = 148 * 1024;       // model + rows; 1 workgroup per CU

// A model's node arrays: the global SoA (feature, dtype apart) or its LDS image
// (feature | dtype << 24 in one word).
struct GbdtGlobal {
  const GbdtParams& p;
  __device__ int node_off(int t) const { return p.node_off[t]; }
  __device__ int leaf_off(int t) const { return p.leaf_off[t]; }
  __device__ int feature(int k) const { return p.feature[k]; }
  __device__ int dtype(int k) const { return p.dtype[k]; }
  __device__ double threshold(int k) const { return p.threshold[k]; }
  __device__ int left(int k) const { return p.left[k]; }
  __device__ int right(int k) const { return p.right[k]; }
  __device__ double leaf(int i) const { return p.leaf_value[i]; }
};
struct GbdtLds {
  const double *thr, *lv;
  const uint32_t* fd;
  const int32_t *lc, *rc, *no, *lo;
  __device__ int node_off(int t) const { return no[t]; }
  __device__ int leaf_off(int t) const { return lo[t]; }
  __device__ int feature(int k) const { return (int)(fd[k] & 0xFFFFFFu); }
  __device__ int dtype(int k) const { return (int)(fd[k] >> 24); }
  __device__ double threshold(int k) const { return thr[k]; }
  __device__ int left(int k) const { return lc[k]; }
  __device__ int right(int k) const { return rc[k]; }
  __device__ double leaf(int i) const { return lv[i]; }
};

template <class M>
__device__ __forceinline__ double gbdt_walk(const M& m, const double* x, int t) {
  const double kZero = (double)1e-35f;  // LightGBM kZeroThreshold (a float)
  const int nb = m.node_off(t), lb = m.leaf_off(t);
  int leaf = 0;
  if (m.leaf_off(t + 1) - lb > 1) {
    int node = 0;
    while (node >= 0) {
      const int k = nb + node;
      double fv = x[m.feature(k)];
      const int dt = m.dtype(k);
      const int missing = (dt >> 2) & 3;  // 0 none, 1 zero, 2 NaN
      if (isnan(fv) && missing != 2) fv = 0.0;
      bool left;
      if ((missing == 1 && fv >= -kZero && fv <= kZero) || (missing == 2 && isnan(fv)))
        left = (dt & 2) != 0;  // default side
      else
        left = fv <= m.threshold(k);
      node = left ? m.left(k) : m.right(k);
    }
    leaf = ~node;
  }
  return m.leaf(lb + leaf);
}

// learned_weights_kernel's arithmetic for one row (lane 0): numpy's clip, the row
// sum as 0.0 + pairwise_sum, the zero guard, the division, 1 / n for unknown runs.
__device__ __forceinline__ void learned_row_weights(const LearnedWeightParams& lw, int64_t q,
                                                    const double* pred) {
  double c[kMaxBoosters];
  for (int b = 0; b < lw.n_boosters; ++b) {
    const double v = pred[b];
    c[b] = (v > 0.0 || isnan(v)) ? v : 0.0;  // np.clip(pred, 0, None): NaN kept, -0.0 -> +0.0
  }
  double s = 0.0 + np_pairwise_sum(c, lw.n_boosters);  // the reduction starts from 0.0
  if (s == 0.0) s = 1.0;
  const double dflt = 1.0 / (double)lw.n_boosters;
  for (int r = 0; r < lw.n_runs; ++r) {
    const int j = lw.run_to_booster[r];
    lw.w_out[q * lw.n_runs + r] = j >= 0 ? c[j] / s : dflt;
  }
}

// A row's features: the X row (qf_gbdt_predict), or read from the QPP micro-units as
// qpp_features_kernel lays them out (qf_learned_gbdt_weights: X[q, 13 j + c] =
// micro[(q R + run[j]) 13 + c] / 1e6, 0.0 for a block without a run).
struct RowFromX {
  const GbdtParams& p;
  __device__ double operator()(int64_t row, int i) const { return p.X[row * p.n_features + i]; }
};
struct RowFromMicro {
  const GbdtFusedParams& f;
  __device__ double operator()(int64_t row, int i) const {
    const int j = i / kQppCols, c = i - j * kQppCols;
    const int r = f.blk.run[j];
    if (r < 0) return 0.0;
    return micro_back(f.micro[(row * f.R + r) * kQppCols + c]);
  }
};
// ... or normalised from the raw predictors on the fly, as qpp_normalize_kernel
// does before its micro-units (no normalisation launch in between).
struct RowFromRaw {
  const GbdtFusedParams& f;
  __device__ double operator()(int64_t row, int i) const {
    const int j = i / kQppCols, c = i - j * kQppCols;
    const int r = f.blk.run[j];
    if (r < 0) return 0.0;
    const int64_t l = row * f.R + r;
    const bool present = f.list_off[l + 1] > f.list_off[l];
    const double m0 = f.norm_mode != 0 ? f.mm[r * kQppCols + c] : 0.0;
    const double m1 = f.norm_mode != 0 ? f.mm[f.R * kQppCols + r * kQppCols + c] : 0.0;
    return micro_back(round6(qpp_norm_value(f.raw_qpp[l * kQppCols + c], m0, m1, f.norm_mode,
                                            present)));
  }
};

// The rows of wave wid, strided over the grid: stage the row, walk, sum; then the
// raw predictions (p.out) and / or the learned weights (lw, when lw->w_out).
template <class M, class X>
__device__ __forceinline__ void gbdt_rows(const GbdtParams& p, const M& m, const X& xrow,
                                          const LearnedWeightParams* lw, double* sxw, double* sl,
                                          int wid, int lane, int T, bool staged) {
  const int b = lane < p.n_boosters ? lane : 0;
  for (int64_t row = (int64_t)blockIdx.x * kGbdtWaves + wid; row < p.n_rows;
       row += (int64_t)gridDim.x * kGbdtWaves) {
    if (staged) {
      for (int i = lane; i < p.n_features; i += 64) sxw[i] = xrow(row, i);
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
    const double* x = staged ? sxw : p.X + row * p.n_features;
    // lane b < n_boosters: booster b's trees [tb, te) and its running sum
    const int tb = p.tree_off[b], te = p.tree_off[b + 1];
    double s = 0.0;
    for (int c0 = 0; c0 < T; c0 += 64) {
      const int t = c0 + lane;
      if (t < T) sl[lane] = gbdt_walk(m, x, t);
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      if (lane < p.n_boosters) {
        const int lo = tb > c0 ? tb : c0, hi = te < c0 + 64 ? te : c0 + 64;
        for (int i = lo; i < hi; ++i) s += sl[i - c0];
      }
      __builtin_amdgcn_wave_barrier();  // every sum read before the next chunk's writes
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
    if (lane < p.n_boosters) {
      if (p.out) p.out[row * p.n_boosters + lane] = s;
      sl[lane] = s;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if (lw && lane == 0) learned_row_weights(*lw, row, sl);
    __builtin_amdgcn_wave_barrier();  // the row's features and sums read before the next row's
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  }
}

// The model's LDS image (when it fits) and the walk of every row; X is the row source.
template <class X>
__device__ __forceinline__ void gbdt_block(const GbdtParams& p, const X& xrow,
                                           const LearnedWeightParams* lw, unsigned char* lds,
                                           double (&sleaf)[kGbdtWaves][64]) {
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int T = p.tree_off[p.n_boosters];
  const int NN = p.node_off[T], NL = p.leaf_off[T], nf = p.n_features;
  const bool staged = nf <= kGbdtMaxFeatures;
  const int64_t xbytes = staged ? (int64_t)8 * kGbdtWaves * nf : 0;
  // LDS image: rows f64 [kGbdtWaves][nf] | thresholds f64 [NN] | leaves f64 [NL] |
  // feature|dtype u32 [NN] | left, right i32 [NN] | node_off, leaf_off i32 [T + 1]
  const int64_t need = xbytes + 8 * (int64_t)NN + 8 * (int64_t)NL + 12 * (int64_t)NN +
                       8 * (int64_t)(T + 1);
  const bool fits = need <= kGbdtLds && nf <= (1 << 24);  // uniform; features fit 24 bits
  double* sx = (double*)lds;
  double* sxw = staged ? sx + (int64_t)wid * nf : nullptr;
  if (fits) {
    double* thr = (double*)(lds + xbytes);
    double* lv = thr + NN;
    uint32_t* fd = (uint32_t*)(lv + NL);
    int32_t* lc = (int32_t*)(fd + NN);
    int32_t* rc = lc + NN;
    int32_t* no = rc + NN;
    int32_t* lo = no + (T + 1);
#pragma unroll 4
    for (int i = tid; i < NN; i += 64 * kGbdtWaves) {
      thr[i] = p.threshold[i];
      // the walk reads decision-type bits 1-3 only: its low byte is kept
      fd[i] = (uint32_t)p.feature[i] | ((uint32_t)(p.dtype[i] & 0xFF) << 24);
      lc[i] = p.left[i];
      rc[i] = p.right[i];
    }
#pragma unroll 4
    for (int i = tid; i < NL; i += 64 * kGbdtWaves) lv[i] = p.leaf_value[i];
    for (int i = tid; i <= T; i += 64 * kGbdtWaves) {
      no[i] = p.node_off[i];
      lo[i] = p.leaf_off[i];
    }
    __syncthreads();
    const GbdtLds m{thr, lv, fd, lc, rc, no, lo};
    gbdt_rows(p, m, xrow, lw, sxw, sleaf[wid], wid, lane, T, staged);
  } else {
    const GbdtGlobal m{p};
    gbdt_rows(p, m, xrow, lw, sxw, sleaf[wid], wid, lane, T, staged);
  }
}

__global__ __launch_bounds__(64 * kGbdtWaves) void gbdt_predict_kernel(GbdtParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[kGbdtLds];
  __shared__ double sleaf[kGbdtWaves][64];
  gbdt_block(p, RowFromX{p}, nullptr, lds, sleaf);
}

// Learned fusion's weights in one launch: features from the QPP micro-units, the
// walk, learned_weights_kernel's normalisation (src/fusion.py:415-440,
// src/models/base.py:120-125) — bit for bit the three-launch path.
__global__ __launch_bounds__(64 * kGbdtWaves) void learned_gbdt_weights_kernel(GbdtFusedParams f) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[kGbdtLds];
  __shared__ double sleaf[kGbdtWaves][64];
  if (f.micro)
    gbdt_block(f.gbdt, RowFromMicro{f}, &f.lw, lds, sleaf);
  else
    gbdt_block(f.gbdt, RowFromRaw{f}, &f.lw, lds, sleaf);
}

__global__ __launch_bounds__(256) void learned_weights_kernel(LearnedWeightParams p) {
  const int64_t q = block_id() * blockDim.x + threadIdx.x;
  if (q >= p.n_queries) return;
  learned_row_weights(p, q, p.pred + q * p.n_boosters);
}

// numpy's float32 pairwise_sum for n < 128 (float32 accumulators)
__device__ __forceinline__ float np_pairwise_sum_f32(const float* a, int n) {
  if (n < 8) {
    float r = 0.0f;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  float r[8];
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}

constexpr int kMlpWaves = 4;  // queries per workgroup (one wave each)

__global__ __launch_bounds__(64 * kMlpWaves) void mlp_weights_kernel(MlpParams p) {
#pragma clang fp contract(off)
  __shared__ float act[kMlpWaves][2][kMlpMaxWidth];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t q = block_id() * kMlpWaves + wid;
  const bool live = q < p.n_queries;  // every wave reaches every barrier
  float* cur = act[wid][0];
  float* nxt = act[wid][1];
  for (int i = lane; i < p.width[0]; i += 64)
    cur[i] = live ? (float)p.X[q * p.x_cols + p.in_col[i]] : 0.0f;  // torch.FloatTensor(X)
  __syncthreads();
  for (int l = 0; l < p.n_layers; ++l) {
    const int n_in = p.width[l], n_o = p.width[l + 1];
    const float* W = p.params + p.w_off[l];
    const float* b = p.params + p.b_off[l];
    const bool relu = l + 1 < p.n_layers;
    for (int o = lane; o < n_o; o += 64) {
      const float* wr = W + (int64_t)o * n_in;
      float acc = 0.0f;
      for (int i = 0; i < n_in; ++i) acc = acc + cur[i] * wr[i];
      acc = acc + b[o];
      if (relu && acc < 0.0f) acc = 0.0f;  // nn.ReLU (NaN passes through)
      nxt[o] = acc;
    }
    __syncthreads();
    float* t = cur;
    cur = nxt;
    nxt = t;
  }
  if (!live || lane != 0) return;
  const int n_out = p.width[p.n_layers];
  float e[kMlpMaxOut];
  float m = cur[0];
  for (int o = 1; o < n_out; ++o) m = fmaxf(m, cur[o]);
  float s = 0.0f;
  for (int o = 0; o < n_out; ++o) {
    e[o] = (float)exp((double)(cur[o] - m));
    s = s + e[o];
  }
  for (int o = 0; o < n_out; ++o) {
    const float v = e[o] / s;
    e[o] = (v > 0.0f || isnan(v)) ? v : 0.0f;  // np.clip(weights, 0, None)
  }
  float sum = 0.0f + np_pairwise_sum_f32(e, n_out);
  if (sum == 0.0f) sum = 1.0f;
  const double dflt = 1.0 / (double)n_out;  // src/fusion.py:440: 1.0 / n_retrievers
  for (int r = 0; r < p.n_runs; ++r) {
    const int j = p.run_to_output[r];
    p.w_out[q * p.n_runs + r] = j >= 0 ? (double)(e[j] / sum) : dflt;
  }
}

hipError_t mlp_weights_launch(const MlpParams& p, hipStream_t st) {
  if (p.n_queries == 0) return hipSuccess;
  hipLaunchKernelGGL(mlp_weights_kernel, grid_for((p.n_queries + kMlpWaves - 1) / kMlpWaves),
                     dim3(64 * kMlpWaves), 0, st, p);
  return hipGetLastError();
}

hipError_t gbdt_predict_launch(const GbdtParams& p, hipStream_t st) {
  if (p.n_rows * p.n_boosters == 0) return hipSuccess;
  // one workgroup per CU at most (its LDS image of the model), each wave striding
  // over the rows
  const int64_t want = (p.n_rows + kGbdtWaves - 1) / kGbdtWaves;
  const unsigned grid = (unsigned)(want < 256 ? want : 256);
  hipLaunchKernelGGL(gbdt_predict_kernel, dim3(grid), dim3(64 * kGbdtWaves), 0, st, p);
  return hipGetLastError();
}

hipError_t learned_gbdt_weights_launch(const GbdtFusedParams& f, hipStream_t st) {
  if (f.gbdt.n_rows == 0) return hipSuccess;
  const int64_t want = (f.gbdt.n_rows + kGbdtWaves - 1) / kGbdtWaves;
  const unsigned grid = (unsigned)(want < 256 ? want : 256);
  hipLaunchKernelGGL(learned_gbdt_weights_kernel, dim3(grid), dim3(64 * kGbdtWaves), 0, st, f);
  return hipGetLastError();
}

hipError_t learned_weights_launch(const LearnedWeightParams& p, hipStream_t st) {
  if (p.n_queries == 0) return hipSuccess;
  hipLaunchKernelGGL(learned_weights_kernel, grid_for((p.n_queries + 255) / 256),
                     dim3(256), 0, st, p);
  return hipGetLastError();
}

}  // namespace qf
