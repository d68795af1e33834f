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

namespace qf {

// One wave per row: the lanes walk the model's trees in parallel (tree c0 + lane
// of each 64-tree chunk, the row's features staged in LDS), then lane b adds
// booster b's leaf values of the chunk in tree order onto its running sum — the
// serial GBDT::PredictRaw sum from 0.0, tree by tree, bit for bit.  (Was: one
// thread per (row, booster) walking its ~30 trees serially — C5: 17,260 threads,
// ~270 waves on 256 CUs, each a chain of ~30 tree walks of dependent loads.)
constexpr int kGbdtWaves = 4;
constexpr int kGbdtMaxFeatures = 256;  // staged in LDS; more features: read from X

__device__ __forceinline__ double gbdt_walk(const GbdtParams& p, const double* x, int t) {
  const double kZero = (double)1e-35f;  // LightGBM kZeroThreshold (a float)
  const int nb = p.node_off[t], lb = p.leaf_off[t];
  int leaf = 0;
  if (p.leaf_off[t + 1] - lb > 1) {
    int node = 0;
    while (node >= 0) {
      const int k = nb + node;
      double fv = x[p.feature[k]];
      const int dt = p.dtype[k];
      const int missing = (dt >> 2) & 3;  // 0 none, 1 zero, 2 NaN
      if (isnan(fv) && missing != 2) fv = 0.0;
      bool left;
      if ((missing == 1 && fv >= -kZero && fv <= kZero) || (missing == 2 && isnan(fv)))
        left = (dt & 2) != 0;  // default side
      else
        left = fv <= p.threshold[k];
      node = left ? p.left[k] : p.right[k];
    }
    leaf = ~node;
  }
  return p.leaf_value[lb + leaf];
}

__global__ __launch_bounds__(64 * kGbdtWaves) void gbdt_predict_kernel(GbdtParams p) {
  __shared__ double sx[kGbdtWaves][kGbdtMaxFeatures];
  __shared__ double sleaf[kGbdtWaves][64];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row = block_id() * kGbdtWaves + wid;
  if (row >= p.n_rows) return;  // whole waves: no block barrier below
  const double* xg = p.X + row * p.n_features;
  const bool staged = p.n_features <= kGbdtMaxFeatures;
  if (staged)
    for (int i = lane; i < p.n_features; i += 64) sx[wid][i] = xg[i];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  const double* x = staged ? sx[wid] : xg;
  const int T = p.tree_off[p.n_boosters];
  // lane b < n_boosters: booster b's trees [tb, te) and its running sum
  const int b = lane < p.n_boosters ? lane : 0;
  const int tb = p.tree_off[b], te = p.tree_off[b + 1];
  double s = 0.0;
  for (int c0 = 0; c0 < T; c0 += 64) {
    const int t = c0 + lane;
    if (t < T) sleaf[wid][lane] = gbdt_walk(p, x, t);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if (lane < p.n_boosters) {
      const int lo = tb > c0 ? tb : c0, hi = te < c0 + 64 ? te : c0 + 64;
      for (int i = lo; i < hi; ++i) s += sleaf[wid][i - c0];
    }
    __builtin_amdgcn_wave_barrier();  // every sum read before the next chunk's writes
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  }
  if (lane < p.n_boosters) p.out[row * p.n_boosters + lane] = s;
}

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

__global__ __launch_bounds__(256) void learned_weights_kernel(LearnedWeightParams p) {
  const int64_t q = block_id() * blockDim.x + threadIdx.x;
  if (q >= p.n_queries) return;
  double c[kMaxBoosters];
  for (int b = 0; b < p.n_boosters; ++b) {
    const double v = p.pred[q * p.n_boosters + b];
    c[b] = (v > 0.0 || isnan(v)) ? v : 0.0;  // np.clip(pred, 0, None): NaN kept, -0.0 -> +0.0
  }
  double s = 0.0 + np_pairwise_sum(c, p.n_boosters);  // the reduction starts from 0.0
  if (s == 0.0) s = 1.0;
  const double dflt = 1.0 / (double)p.n_boosters;
  for (int r = 0; r < p.n_runs; ++r) {
    const int j = p.run_to_booster[r];
    p.w_out[q * p.n_runs + r] = j >= 0 ? c[j] / s : dflt;
  }
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
  hipLaunchKernelGGL(gbdt_predict_kernel, grid_for((p.n_rows + kGbdtWaves - 1) / kGbdtWaves),
                     dim3(64 * kGbdtWaves), 0, st, p);
  return hipGetLastError();
}

hipError_t learned_weights_launch(const LearnedWeightParams& p, hipStream_t st) {
  if (p.n_queries == 0) return hipSuccess;
  hipLaunchKernelGGL(learned_weights_kernel, grid_for((p.n_queries + 255) / 256),
                     dim3(256), 0, st, p);
  return hipGetLastError();
}

}  // namespace qf
