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
// gbdt_predict_kernel — one thread per (row, booster): walks that booster's
//   first best_iteration trees (LightGBM NumericalDecision; see qppfuse/lgbm.py)
//   and adds the leaf values in tree order from 0.0, as GBDT::PredictRaw does.
//   The model (≈4.5 k nodes for the reference's NQ model) stays in L1/L2.
// learned_weights_kernel — one thread per query: numpy's clip (NaN kept, -0.0
//   becomes +0.0 — measured on numpy 2.2), numpy's row sum (0.0 + pairwise_sum: sequential below 8
//   values, 8 accumulators from 8), the zero guard and the division.
#include <math.h>

#include "../../include/qppfuse.h"
#include "qf_common.h"
#include "qf_internal.h"

namespace qf {

__global__ __launch_bounds__(256) void gbdt_predict_kernel(GbdtParams p) {
  const int64_t idx = block_id() * blockDim.x + threadIdx.x;
  if (idx >= p.n_rows * p.n_boosters) return;
  const int64_t row = idx / p.n_boosters;
  const int b = (int)(idx % p.n_boosters);
  const double* x = p.X + row * p.n_features;
  const double kZero = (double)1e-35f;  // LightGBM kZeroThreshold (a float)
  double s = 0.0;
  for (int t = p.tree_off[b]; t < p.tree_off[b + 1]; ++t) {
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
    s += p.leaf_value[lb + leaf];
  }
  p.out[idx] = s;
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

hipError_t gbdt_predict_launch(const GbdtParams& p, hipStream_t st) {
  const int64_t n = p.n_rows * p.n_boosters;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(gbdt_predict_kernel, grid_for((n + 255) / 256), dim3(256), 0, st, p);
  return hipGetLastError();
}

hipError_t learned_weights_launch(const LearnedWeightParams& p, hipStream_t st) {
  if (p.n_queries == 0) return hipSuccess;
  hipLaunchKernelGGL(learned_weights_kernel, grid_for((p.n_queries + 255) / 256),
                     dim3(256), 0, st, p);
  return hipGetLastError();
}

}  // namespace qf
