// qf_internal.h — launcher declarations shared by the kernel files and the C-ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qf {

// A grid of n_blocks workgroups.  A dispatch holds at most 2^32 - 1 work-items per
// dimension (a C3-sized synth or a 10-million-query join exceeds that in x alone),
// so beyond 65,536 workgroups the grid folds into y; kernels take block_id() and
// return for ids >= n_blocks (the last y row may overshoot).
inline dim3 grid_for(int64_t n_blocks) {
  if (n_blocks <= 65536) return dim3((unsigned)(n_blocks > 0 ? n_blocks : 1));
  return dim3(65536u, (unsigned)((n_blocks + 65535) / 65536));
}


struct FuseParams {
  int64_t n_queries;
  int32_t R;
  const int64_t* list_off;
  const uint32_t* docid;
  const void* score;
  const int32_t* rank;
  const double* weights;
  int32_t methods;
  int32_t rrf_k;
  uint32_t* union_docid;
  int32_t* union_count;
  void* perm;      // uint16 [M][E], or uint32 when perm32 (qf_fuse_wide)
  double* fused;
  int64_t out_stride;
  const double* seg_prob;  // QF_PROBFUSE: [R][n_seg] segment probabilities
  int32_t n_seg, seg_len;  // x and L of ProbFuse.py
  // QF_LEARNED with FusionMLP's float32 weights (qf_fuse_learned_f32): bit r set =
  // run r's products are float32; learned_sum_f32 = the groupby sum is float32 Kahan
  uint32_t learned_f32;
  int32_t learned_sum_f32;
  int32_t perm32;  // perm holds uint32 entries (unions above 65,535 documents)
  // qf_fuse_qpp: the W-* weights from the raw QPP predictors [Q*R][13] and their
  // column statistics [2][R][13] (QF_NORM_* qpp_mode), column qpp_index (-1: the
  // mean of the 13) — qf_qpp_normalize's w_out computed in the join; NULL: weights
  const double* qpp_raw;
  const double* qpp_stats;
  int32_t qpp_mode, qpp_index;
  // the largest union learned fusion's bucket sort reaches in this call (0: kJsUMax);
  // the fallback pass takes a learned pair above it or marked below it
  int32_t learned_reach;
  // the largest union the other slots' bucket sorts reach in this call (0: kJsUMax —
  // the 1,024-thread configuration not launched); the fallback pass takes a pair
  // above it, or marked below it
  int32_t fast_reach;
  // qf_fuse_qpp_micro: the join also writes the .qpp "%.6f" micro-units of all 13
  // normalised columns of its query's lists ([Q*R][13], qf_qpp_normalize's micro_out)
  int64_t* qpp_micro;
};
// perm element i (m * out_stride + base + rank): every kernel writes perm through
// these, so one flag switches a call between the uint16 and uint32 layouts
__device__ __forceinline__ void perm_put(const FuseParams& p, int64_t i, uint32_t u) {
  if (p.perm32) __builtin_nontemporal_store(u, (uint32_t*)p.perm + i);
  else __builtin_nontemporal_store((uint16_t)u, (uint16_t*)p.perm + i);
}
__device__ __forceinline__ uint32_t perm_get(const FuseParams& p, int64_t i) {
  return p.perm32 ? ((const uint32_t*)p.perm)[i] : ((const uint16_t*)p.perm)[i];
}

// IR evaluation (qf_eval): run m, query q reads its ranked list at
// [q_base[q*base_stride], + q_count[q] (or up to the next base)) of score /
// perm (+ m*out_stride) and docid (shared through perm, else + m*out_stride).
constexpr int kEvalMaxRel = 256;  // judged documents per query
constexpr int kEvalMaxMetrics = 16;
struct EvalParams {
  int64_t n_queries;
  const int64_t* q_base;
  int32_t base_stride;
  const int32_t* q_count;
  const uint32_t* docid;
  const uint16_t* perm;
  const double* score;
  int64_t out_stride;
  int32_t n_runs;
  int32_t text_scores;
  const int64_t* qrel_off;
  const uint32_t* qrel_docid;
  const int32_t* qrel_rel;
  int32_t n_metrics;
  int32_t kind[kEvalMaxMetrics];
  int32_t cut[kEvalMaxMetrics];
  double* out;
};

// LightGBM inference (qf_gbdt_predict) and learned weights (qf_learned_weights).
constexpr int kMaxBoosters = 16;
constexpr int kMaxLearnedRuns = 32;  // runs a learned weight table maps (qf_fuse's run cap)
struct GbdtParams {
  int64_t n_rows;
  const double* X;
  int32_t n_features;
  int32_t n_boosters;
  const int32_t* tree_off;
  const int32_t* node_off;
  const int32_t* leaf_off;
  const int32_t* feature;
  const double* threshold;
  const int32_t* dtype;
  const int32_t* left;
  const int32_t* right;
  const double* leaf_value;
  double* out;
};
struct LearnedWeightParams {
  int64_t n_queries;
  const double* pred;
  int32_t n_boosters;
  int32_t n_runs;
  int32_t run_to_booster[kMaxLearnedRuns];
  double* w_out;
};
constexpr int kMaxFeatureBlocks = 32;  // model retrievers of a learned-fusion feature matrix
struct QppBlocks {
  int32_t n;
  int32_t run[kMaxFeatureBlocks];
};
// qf_learned_gbdt_weights: the feature matrix read from the QPP micro-units as
// qpp_features_kernel builds it, the GBDT walk, and the weights as
// learned_weights_kernel computes them, in one launch (gbdt.X unused; gbdt.out
// nullable: the raw predictions, if wanted).
struct GbdtFusedParams {
  GbdtParams gbdt;
  const int64_t* micro;  // [n_rows * R][13] QPP micro-units (qf_qpp_normalize), or NULL:
  const double* raw_qpp;   // [n_rows * R][13] raw predictors, normalised on the fly with
  const double* mm;        // the column statistics (qf_qpp_colminmax / colmeanstd)
  const int64_t* list_off;  // (absent lists: 0.0)
  int32_t norm_mode;       // QF_NORM_*
  int32_t R;
  QppBlocks blk;
  LearnedWeightParams lw;  // lw.pred unused; lw.w_out [n_rows][n_runs]
};
hipError_t gbdt_predict_launch(const GbdtParams& p, hipStream_t st);
hipError_t learned_gbdt_weights_launch(const GbdtFusedParams& p, hipStream_t st);
hipError_t learned_weights_launch(const LearnedWeightParams& p, hipStream_t st);

// FusionMLP inference + weights (qf_mlp_weights): Linear layers (ReLU between,
// Dropout = identity in eval), softmax, _normalize_weights, all in float32.
constexpr int kMlpMaxLayers = 8;
constexpr int kMlpMaxWidth = 512;  // inputs and every layer's width
constexpr int kMlpMaxOut = 32;     // retrievers the model predicts weights for
struct MlpParams {
  int64_t n_queries;
  const double* X;        // [n_queries][x_cols] the learned_fusion feature matrix
  int32_t x_cols;
  const int32_t* in_col;  // [width[0]] column of X feeding model input i
  int32_t n_layers;
  int32_t width[kMlpMaxLayers + 1];
  int64_t w_off[kMlpMaxLayers];  // layer l: W [width[l+1]][width[l]] at params + w_off[l],
  int64_t b_off[kMlpMaxLayers];  //          b [width[l+1]] at params + b_off[l]
  const float* params;
  int32_t n_runs;
  int32_t run_to_output[kMaxLearnedRuns];
  double* w_out;  // [n_queries][n_runs]
};
hipError_t mlp_weights_launch(const MlpParams& p, hipStream_t st);

int fuse_max_entries(int wide);
hipError_t eval_launch(const EvalParams& p, hipStream_t st);
// ws_user (nullable): the caller's workspace of ws_bytes for the workspace kernel;
// NULL = stream-ordered allocation (hipMallocAsync / hipFreeAsync on st)
hipError_t fuse_launch(const FuseParams& p, int kind, int max_entries, hipStream_t st,
                       void* ws_user = nullptr, size_t ws_bytes = 0);
// Bytes of the workspace fuse_launch would allocate (0: no workspace kernel);
// *min_bytes: the least a caller's workspace may hold (one workgroup's share).
int64_t fuse_workspace_bytes(int64_t n_queries, int R, int max_entries, int perm32,
                             int64_t* min_bytes);
hipError_t topk_launch(int64_t n_queries, int32_t R, const int64_t* list_off,
                       const int32_t* union_count, const uint32_t* union_docid,
                       const void* perm, int perm32, const double* fused, int64_t out_stride,
                       int32_t M, int32_t k, uint32_t* out_docid, double* out_score,
                       hipStream_t st);
hipError_t qpp_raw_launch(const double* score, const int64_t* list_off, int64_t Q, int32_t R,
                          int32_t top_k, const int32_t* nt, const double* tf, double* out,
                          hipStream_t st);
hipError_t qpp_colminmax_launch(const double* raw, const int64_t* list_off, int64_t Q, int32_t R,
                                double* mm, hipStream_t st);
hipError_t qpp_colmeanstd_launch(const double* raw, const int64_t* list_off, int64_t Q,
                                 int32_t R, double* st, hipStream_t stm);
hipError_t qpp_features_launch(const int64_t* micro, int64_t Q, int32_t R, const QppBlocks& blk,
                               double* X, hipStream_t st);
hipError_t qpp_normalize_launch(const double* raw, const double* mm, const int64_t* list_off,
                                int64_t Q, int32_t R, int32_t mode, int32_t qpp_index,
                                double* norm_out, int64_t* micro_out, double* w_out,
                                hipStream_t st);
hipError_t minmax_colminmax_launch(const double* score, const int64_t* list_off, int64_t Q,
                                   int32_t R, double* out_norm, int32_t* out_micro,
                                   const double* raw, double* mm, hipStream_t st);
hipError_t minmax_launch(const double* score, const int64_t* list_off, int64_t n_lists,
                         double* out_norm, int32_t* out_micro, hipStream_t st);
hipError_t stream_copy_launch(void* dst, const void* src, int64_t n16, hipStream_t st);
hipError_t synth_nq_launch(int64_t q_begin, int64_t n_queries, int32_t R, int32_t K,
                           uint64_t seed, const int64_t* qrel_off, const uint32_t* qrel_doc,
                           int64_t n_qrel_q, int64_t* list_off, uint32_t* docid, double* score,
                           hipStream_t st);
hipError_t synth_launch(int64_t q_begin, int64_t n_queries, int32_t R, int32_t K, uint64_t seed,
                        double p_shared, int64_t* list_off, uint32_t* docid, double* score,
                        hipStream_t st);

}  // namespace qf
