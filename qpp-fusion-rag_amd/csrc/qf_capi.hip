// qf_capi.hip — the C-ABI of libqppfuse.so (declared in include/qppfuse.h).
// Argument validation, kernel selection, thread-local error strings.  No entry
// point synchronises: everything is stream-ordered on the caller's stream.  The
// only allocation is qf_fuse's workspace for queries beyond the LDS join (more
// than 10,240 entries or 16 runs): hipMallocAsync / hipFreeAsync on the call's
// stream (include/qppfuse.h).
#include <cstdio>
#include <string>

#include "../../include/qppfuse.h"
#include "qf_internal.h"
#include <cstdarg>


namespace {
thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int check(hipError_t e, const char* what) {
  if (e != hipSuccess) return fail(QF_EHIP, "%s: %s", what, hipGetErrorString(e));
  g_err.clear();
  return QF_OK;
}

constexpr int kMaxR = 32;  // qf_fuse: > 16 runs take the workspace kernel
constexpr int kMaxRLds = 16;  // runs of the LDS join (qf_fuse_qpp_micro's values are its)
}  // namespace

extern "C" {

const char* qf_version(void) { return "qppfuse 0.1.0 gfx950"; }
const char* qf_last_error(void) { return g_err.c_str(); }
int qf_max_entries_per_query(void) { return qf::fuse_max_entries(0); }
int qf_max_entries_per_query_wide(void) { return qf::fuse_max_entries(1); }

int qf_minmax_per_query(const double* score, const int64_t* list_off, int64_t n_lists,
                        double* out_norm, int32_t* out_micro, void* stream) {
  if (n_lists < 0 || (n_lists > 0 && (!score || !list_off)))
    return fail(QF_EINVAL, "qf_minmax_per_query: bad arguments");
  if (!out_norm && !out_micro) return fail(QF_EINVAL, "qf_minmax_per_query: no output");
  return check(qf::minmax_launch(score, list_off, n_lists, out_norm, out_micro,
                                 (hipStream_t)stream),
               "qf_minmax_per_query");
}

int qf_qpp_raw(const double* score, const int64_t* list_off, int64_t n_queries,
               int32_t n_retrievers, int32_t top_k, const int32_t* num_terms,
               const double* text_feat, double* raw_out, void* stream) {
  if (n_queries < 0 || n_retrievers <= 0 || !list_off || !num_terms || !text_feat || !raw_out ||
      (!score && n_queries > 0))
    return fail(QF_EINVAL, "qf_qpp_raw: bad arguments");
  return check(qf::qpp_raw_launch(score, list_off, n_queries, n_retrievers, top_k, num_terms,
                                  text_feat, raw_out, (hipStream_t)stream),
               "qf_qpp_raw");
}

int qf_qpp_colminmax(const double* raw, const int64_t* list_off, int64_t n_queries,
                     int32_t n_retrievers, double* mm_out, void* stream) {
  if (n_queries < 0 || n_retrievers <= 0 || !raw || !list_off || !mm_out)
    return fail(QF_EINVAL, "qf_qpp_colminmax: bad arguments");
  return check(qf::qpp_colminmax_launch(raw, list_off, n_queries, n_retrievers, mm_out,
                                        (hipStream_t)stream),
               "qf_qpp_colminmax");
}

int qf_minmax_colminmax(const double* score, const int64_t* list_off, int64_t n_queries,
                        int32_t n_retrievers, double* out_norm, int32_t* out_micro,
                        const double* raw_qpp, double* mm_out, void* stream) {
  if (n_queries < 0 || n_retrievers <= 0 || !list_off || !raw_qpp || !mm_out ||
      (n_queries > 0 && !score))
    return fail(QF_EINVAL, "qf_minmax_colminmax: bad arguments");
  if (!out_norm && !out_micro) return fail(QF_EINVAL, "qf_minmax_colminmax: no output");
  return check(qf::minmax_colminmax_launch(score, list_off, n_queries, n_retrievers, out_norm,
                                           out_micro, raw_qpp, mm_out, (hipStream_t)stream),
               "qf_minmax_colminmax");
}

int qf_qpp_colmeanstd(const double* raw, const int64_t* list_off, int64_t n_queries,
                      int32_t n_retrievers, double* st_out, void* stream) {
  if (n_queries < 0 || n_retrievers <= 0 || !raw || !list_off || !st_out)
    return fail(QF_EINVAL, "qf_qpp_colmeanstd: bad arguments");
  return check(qf::qpp_colmeanstd_launch(raw, list_off, n_queries, n_retrievers, st_out,
                                         (hipStream_t)stream),
               "qf_qpp_colmeanstd");
}

int qf_qpp_normalize(const double* raw, const double* mm, const int64_t* list_off,
                     int64_t n_queries, int32_t n_retrievers, int32_t mode, int32_t qpp_index,
                     double* norm_out, int64_t* micro_out, double* w_out, void* stream) {
  if (n_queries < 0 || n_retrievers <= 0 || !raw || !list_off || (mode != QF_NORM_NONE && !mm))
    return fail(QF_EINVAL, "qf_qpp_normalize: bad arguments");
  if (mode != QF_NORM_NONE && mode != QF_NORM_MINMAX && mode != QF_NORM_ZSCORE)
    return fail(QF_EINVAL, "qf_qpp_normalize: unsupported mode %d", mode);
  if (qpp_index < -1 || qpp_index >= QF_QPP_COLS)
    return fail(QF_EINVAL, "qf_qpp_normalize: qpp_index %d out of range", qpp_index);
  return check(qf::qpp_normalize_launch(raw, mm, list_off, n_queries, n_retrievers, mode,
                                        qpp_index, norm_out, micro_out, w_out,
                                        (hipStream_t)stream),
               "qf_qpp_normalize");
}

int qf_qpp_features(const int64_t* micro, int64_t n_queries, int32_t n_retrievers,
                    const int32_t* run_of_block, int32_t n_blocks, double* X, void* stream) {
  if (n_queries < 0 || n_retrievers <= 0 || n_blocks <= 0 || n_blocks > qf::kMaxFeatureBlocks ||
      !run_of_block || (n_queries > 0 && (!micro || !X)))
    return fail(QF_EINVAL, "qf_qpp_features: bad arguments (n_blocks must be in [1, %d])",
                qf::kMaxFeatureBlocks);
  qf::QppBlocks blk{};
  blk.n = n_blocks;
  for (int j = 0; j < n_blocks; ++j) {
    if (run_of_block[j] < -1 || run_of_block[j] >= n_retrievers)
      return fail(QF_EINVAL, "qf_qpp_features: run_of_block[%d] = %d out of range", j,
                  run_of_block[j]);
    blk.run[j] = run_of_block[j];
  }
  return check(qf::qpp_features_launch(micro, n_queries, n_retrievers, blk, X,
                                       (hipStream_t)stream),
               "qf_qpp_features");
}

static int fuse_common(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
                       const uint32_t* docid, const void* score, int32_t score_kind,
                       const int32_t* rank, const double* weights, int32_t methods,
                       int32_t rrf_k, const double* seg_prob, int32_t n_seg, int32_t seg_len,
                       int32_t max_entries, uint32_t* union_docid, int32_t* union_count,
                       void* perm, int perm32, double* fused, int64_t out_stride,
                       void* stream, const char* fn, uint32_t learned_f32 = 0u,
                       void* ws = nullptr, size_t ws_bytes = 0,
                       const double* qpp_raw = nullptr, const double* qpp_stats = nullptr,
                       int32_t qpp_mode = 0, int32_t qpp_index = -1,
                       int64_t* qpp_micro = nullptr) {
  if (n_queries < 0 || n_retrievers <= 0 || n_retrievers > kMaxR)
    return fail(QF_EINVAL, "%s: n_retrievers must be in [1, %d]", fn, kMaxR);
  if (methods <= 0 ||
      (methods & ~(QF_ALL_METHODS | QF_LEARNED | QF_PROBFUSE | QF_WRRF_MUL)))
    return fail(QF_EINVAL, "%s: bad method mask 0x%x", fn, methods);
  if ((methods & (QF_WCOMBSUM | QF_WCOMBMNZ | QF_WRRF | QF_LEARNED | QF_WRRF_MUL)) && !weights &&
      !qpp_raw)
    return fail(QF_EINVAL, "%s: weighted method requested without weights", fn);
  if (qpp_raw && (methods & QF_LEARNED))
    return fail(QF_EINVAL, "%s: QF_LEARNED takes its learned weights, not QPP ones", fn);
  if (qpp_raw && (qpp_index < -1 || qpp_index >= QF_QPP_COLS ||
                  (qpp_mode != QF_NORM_NONE && qpp_mode != QF_NORM_MINMAX &&
                   qpp_mode != QF_NORM_ZSCORE) ||
                  (qpp_mode != QF_NORM_NONE && !qpp_stats)))
    return fail(QF_EINVAL, "%s: bad QPP weight arguments (index %d, mode %d)", fn, qpp_index,
                qpp_mode);
  if ((methods & QF_LEARNED) && (methods & (QF_WCOMBSUM | QF_WCOMBMNZ | QF_WRRF | QF_WRRF_MUL)))
    return fail(QF_EINVAL, "%s: QF_LEARNED and the W-* methods need different weights", fn);
  if ((methods & QF_PROBFUSE) && (!seg_prob || n_seg <= 0 || seg_len <= 0))
    return fail(QF_EINVAL, "%s: QF_PROBFUSE needs the segment table, x > 0 and L > 0", fn);
  if (score_kind != QF_SCORE_F64 && score_kind != QF_SCORE_MICRO)
    return fail(QF_EINVAL, "%s: bad score_kind %d", fn, score_kind);
  if (max_entries > qf::fuse_max_entries(perm32))
    return fail(QF_ETOOBIG, "%s: %d entries in one query exceed the kernel limit %d%s", fn,
                max_entries, qf::fuse_max_entries(perm32),
                perm32 ? "" : " (the _wide entry points take more, with a uint32 perm)");
  if (n_queries == 0) return QF_OK;
  if (!list_off || !docid || !score || !union_docid || !union_count || !perm || !fused ||
      out_stride < 0)
    return fail(QF_EINVAL, "%s: null buffer", fn);
  qf::FuseParams p{n_queries, n_retrievers, list_off,    docid,       score, rank,
                   weights,   methods,      rrf_k,       union_docid, union_count,
                   perm,      fused,        out_stride,  seg_prob,    n_seg, seg_len};
  p.perm32 = perm32;
  p.qpp_raw = qpp_raw;
  p.qpp_stats = qpp_stats;
  p.qpp_mode = qpp_mode;
  p.qpp_index = qpp_index;
  p.qpp_micro = qpp_micro;
  if (learned_f32) {
    const uint32_t all = n_retrievers == 32 ? 0xFFFFFFFFu : (1u << n_retrievers) - 1u;
    p.learned_f32 = learned_f32 & all;
    p.learned_sum_f32 = (learned_f32 & all) == all;
  }
  if (ws) {
    // each workgroup's share (a multiple of 256 bytes) holds the hash table's u32
    // atomicCAS targets and u64 sort words: the base must be 256-byte aligned
    if ((uintptr_t)ws % 256u != 0u)
      return fail(QF_EINVAL, "%s: workspace %p is not 256-byte aligned", fn, ws);
    int64_t min_bytes = 0;
    qf::fuse_workspace_bytes(n_queries, n_retrievers, max_entries, perm32, &min_bytes);
    if ((int64_t)ws_bytes < min_bytes)
      return fail(QF_EINVAL, "%s: workspace of %zu bytes, at least %lld needed", fn, ws_bytes,
                  (long long)min_bytes);
  }
  return check(qf::fuse_launch(p, score_kind, max_entries < 1 ? 1 : max_entries,
                               (hipStream_t)stream, ws, ws_bytes),
               fn);
}

int qf_fuse(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
            const uint32_t* docid, const void* score, int32_t score_kind, const int32_t* rank,
            const double* weights, int32_t methods, int32_t rrf_k, int32_t max_entries,
            uint32_t* union_docid, int32_t* union_count, uint16_t* perm, double* fused,
            int64_t out_stride, void* stream) {
  if (methods & QF_PROBFUSE)
    return fail(QF_EINVAL, "qf_fuse: QF_PROBFUSE needs qf_fuse_probfuse (segment table)");
  return fuse_common(n_queries, n_retrievers, list_off, docid, score, score_kind, rank, weights,
                     methods, rrf_k, nullptr, 0, 0, max_entries, union_docid, union_count, perm,
                     0, fused, out_stride, stream, "qf_fuse");
}

int qf_fuse_qpp(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
                const uint32_t* docid, const void* score, int32_t score_kind, const int32_t* rank,
                const double* qpp_raw, const double* qpp_stats, int32_t qpp_mode,
                int32_t qpp_index, int32_t methods, int32_t rrf_k, int32_t max_entries,
                uint32_t* union_docid, int32_t* union_count, uint16_t* perm, double* fused,
                int64_t out_stride, void* stream) {
  if (methods & QF_PROBFUSE)
    return fail(QF_EINVAL, "qf_fuse_qpp: QF_PROBFUSE needs qf_fuse_probfuse (segment table)");
  if (n_queries > 0 && !qpp_raw) return fail(QF_EINVAL, "qf_fuse_qpp: null buffer");
  return fuse_common(n_queries, n_retrievers, list_off, docid, score, score_kind, rank, nullptr,
                     methods, rrf_k, nullptr, 0, 0, max_entries, union_docid, union_count, perm,
                     0, fused, out_stride, stream, "qf_fuse_qpp", 0u, nullptr, 0, qpp_raw,
                     qpp_stats, qpp_mode, qpp_index);
}

int qf_fuse_qpp_micro(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
                      const uint32_t* docid, const void* score, int32_t score_kind,
                      const int32_t* rank, const double* qpp_raw, const double* qpp_stats,
                      int32_t qpp_mode, int32_t qpp_index, int32_t methods, int32_t rrf_k,
                      int32_t max_entries, uint32_t* union_docid, int32_t* union_count,
                      uint16_t* perm, double* fused, int64_t out_stride, int64_t* qpp_micro_out,
                      void* stream) {
  if (methods & QF_PROBFUSE)
    return fail(QF_EINVAL, "qf_fuse_qpp_micro: QF_PROBFUSE needs qf_fuse_probfuse (segment table)");
  if (n_queries > 0 && (!qpp_raw || !qpp_micro_out))
    return fail(QF_EINVAL, "qf_fuse_qpp_micro: null buffer");
  if (n_retrievers > kMaxRLds)  // the workspace join of 17-32 runs writes none
    return fail(QF_EINVAL, "qf_fuse_qpp_micro: at most %d runs", kMaxRLds);
  return fuse_common(n_queries, n_retrievers, list_off, docid, score, score_kind, rank, nullptr,
                     methods, rrf_k, nullptr, 0, 0, max_entries, union_docid, union_count, perm,
                     0, fused, out_stride, stream, "qf_fuse_qpp_micro", 0u, nullptr, 0, qpp_raw,
                     qpp_stats, qpp_mode, qpp_index, qpp_micro_out);
}

int64_t qf_fuse_workspace_bytes(int64_t n_queries, int32_t n_retrievers, int32_t max_entries,
                                int32_t methods, int32_t wide) {
  (void)methods;  // every method shares the one workspace per workgroup
  if (n_queries <= 0 || n_retrievers <= 0 || n_retrievers > kMaxR || max_entries < 0 ||
      max_entries > qf::fuse_max_entries(wide ? 1 : 0))
    return 0;
  return qf::fuse_workspace_bytes(n_queries, n_retrievers, max_entries, wide ? 1 : 0, nullptr);
}

int qf_fuse_ws(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
               const uint32_t* docid, const void* score, int32_t score_kind, const int32_t* rank,
               const double* weights, int32_t methods, int32_t rrf_k, int32_t max_entries,
               uint32_t* union_docid, int32_t* union_count, void* perm, int32_t wide,
               double* fused, int64_t out_stride, void* ws, size_t ws_bytes, void* stream) {
  if (methods & QF_PROBFUSE)
    return fail(QF_EINVAL, "qf_fuse_ws: QF_PROBFUSE needs qf_fuse_probfuse (segment table)");
  return fuse_common(n_queries, n_retrievers, list_off, docid, score, score_kind, rank, weights,
                     methods, rrf_k, nullptr, 0, 0, max_entries, union_docid, union_count, perm,
                     wide ? 1 : 0, fused, out_stride, stream, "qf_fuse_ws", 0u, ws, ws_bytes);
}

int qf_fuse_wide(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
                 const uint32_t* docid, const void* score, int32_t score_kind, const int32_t* rank,
                 const double* weights, int32_t methods, int32_t rrf_k, int32_t max_entries,
                 uint32_t* union_docid, int32_t* union_count, uint32_t* perm, double* fused,
                 int64_t out_stride, void* stream) {
  if (methods & QF_PROBFUSE)
    return fail(QF_EINVAL, "qf_fuse_wide: QF_PROBFUSE needs qf_fuse_probfuse_wide (segment table)");
  return fuse_common(n_queries, n_retrievers, list_off, docid, score, score_kind, rank, weights,
                     methods, rrf_k, nullptr, 0, 0, max_entries, union_docid, union_count, perm,
                     1, fused, out_stride, stream, "qf_fuse_wide");
}

int qf_fuse_probfuse(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
                     const uint32_t* docid, const void* score, int32_t score_kind,
                     const int32_t* rank, const double* weights, int32_t methods,
                     int32_t rrf_k, const double* seg_prob, int32_t n_segments,
                     int32_t seg_len, int32_t max_entries, uint32_t* union_docid,
                     int32_t* union_count, uint16_t* perm, double* fused, int64_t out_stride,
                     void* stream) {
  return fuse_common(n_queries, n_retrievers, list_off, docid, score, score_kind, rank, weights,
                     methods, rrf_k, seg_prob, n_segments, seg_len, max_entries, union_docid,
                     union_count, perm, 0, fused, out_stride, stream, "qf_fuse_probfuse");
}

int qf_fuse_probfuse_wide(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
                          const uint32_t* docid, const void* score, int32_t score_kind,
                          const int32_t* rank, const double* weights, int32_t methods,
                          int32_t rrf_k, const double* seg_prob, int32_t n_segments,
                          int32_t seg_len, int32_t max_entries, uint32_t* union_docid,
                          int32_t* union_count, uint32_t* perm, double* fused,
                          int64_t out_stride, void* stream) {
  return fuse_common(n_queries, n_retrievers, list_off, docid, score, score_kind, rank, weights,
                     methods, rrf_k, seg_prob, n_segments, seg_len, max_entries, union_docid,
                     union_count, perm, 1, fused, out_stride, stream, "qf_fuse_probfuse_wide");
}

int qf_fuse_learned_f32(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
                        const uint32_t* docid, const void* score, int32_t score_kind,
                        const double* weights, uint32_t f32_runs, int32_t max_entries,
                        uint32_t* union_docid, int32_t* union_count, uint16_t* perm,
                        double* fused, int64_t out_stride, void* stream) {
  return fuse_common(n_queries, n_retrievers, list_off, docid, score, score_kind, nullptr,
                     weights, QF_LEARNED, 60, nullptr, 0, 0, max_entries, union_docid,
                     union_count, perm, 0, fused, out_stride, stream, "qf_fuse_learned_f32",
                     f32_runs);
}

int qf_fuse_learned_f32_wide(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
                             const uint32_t* docid, const void* score, int32_t score_kind,
                             const double* weights, uint32_t f32_runs, int32_t max_entries,
                             uint32_t* union_docid, int32_t* union_count, uint32_t* perm,
                             double* fused, int64_t out_stride, void* stream) {
  return fuse_common(n_queries, n_retrievers, list_off, docid, score, score_kind, nullptr,
                     weights, QF_LEARNED, 60, nullptr, 0, 0, max_entries, union_docid,
                     union_count, perm, 1, fused, out_stride, stream,
                     "qf_fuse_learned_f32_wide", f32_runs);
}

static int topk_common(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
                       const int32_t* union_count, const uint32_t* union_docid, const void* perm,
                       int perm32, const double* fused, int64_t out_stride, int32_t n_methods,
                       int32_t k, uint32_t* out_docid, double* out_score, void* stream,
                       const char* fn) {
  if (n_queries < 0 || n_retrievers <= 0 || n_methods <= 0 || k < 0 || out_stride < 0)
    return fail(QF_EINVAL, "%s: bad sizes", fn);
  if (n_queries > 0 && k > 0 &&
      (!list_off || !union_count || !union_docid || !perm || !fused || !out_docid || !out_score))
    return fail(QF_EINVAL, "%s: null buffer", fn);
  return check(qf::topk_launch(n_queries, n_retrievers, list_off, union_count, union_docid, perm,
                               perm32, fused, out_stride, n_methods, k, out_docid, out_score,
                               (hipStream_t)stream),
               fn);
}

int qf_fused_topk(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
                  const int32_t* union_count, const uint32_t* union_docid, const uint16_t* perm,
                  const double* fused, int64_t out_stride, int32_t n_methods, int32_t k,
                  uint32_t* out_docid, double* out_score, void* stream) {
  return topk_common(n_queries, n_retrievers, list_off, union_count, union_docid, perm, 0, fused,
                     out_stride, n_methods, k, out_docid, out_score, stream, "qf_fused_topk");
}

int qf_fused_topk_wide(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
                       const int32_t* union_count, const uint32_t* union_docid,
                       const uint32_t* perm, const double* fused, int64_t out_stride,
                       int32_t n_methods, int32_t k, uint32_t* out_docid, double* out_score,
                       void* stream) {
  return topk_common(n_queries, n_retrievers, list_off, union_count, union_docid, perm, 1, fused,
                     out_stride, n_methods, k, out_docid, out_score, stream,
                     "qf_fused_topk_wide");
}

int qf_eval(int64_t n_queries, const int64_t* q_base, int32_t base_stride,
            const int32_t* q_count, const uint32_t* docid, const uint16_t* perm,
            const double* score, int64_t out_stride, int32_t n_runs, int32_t text_scores,
            const int64_t* qrel_off, const uint32_t* qrel_docid, const int32_t* qrel_rel,
            int32_t max_qrels, int32_t n_metrics, const int32_t* kind, const int32_t* cut,
            double* out, void* stream) {
  if (n_queries < 0 || n_runs < 0 || base_stride <= 0 || out_stride < 0)
    return fail(QF_EINVAL, "qf_eval: bad sizes");
  if (n_metrics <= 0 || n_metrics > QF_EVAL_MAX_METRICS || !kind || !cut)
    return fail(QF_EINVAL, "qf_eval: n_metrics must be in [1, %d]", QF_EVAL_MAX_METRICS);
  if (max_qrels < 0 || max_qrels > QF_EVAL_MAX_QRELS)
    return fail(QF_ETOOBIG, "qf_eval: %d judged documents in one query exceed %d", max_qrels,
                QF_EVAL_MAX_QRELS);
  qf::EvalParams p{};
  for (int t = 0; t < n_metrics; ++t) {
    if (kind[t] < QF_EVAL_NDCG || kind[t] > QF_EVAL_AP)
      return fail(QF_EINVAL, "qf_eval: bad metric kind %d", kind[t]);
    if (kind[t] != QF_EVAL_AP && cut[t] < 1)
      return fail(QF_EINVAL, "qf_eval: metric cutoff must be >= 1");
    p.kind[t] = kind[t];
    p.cut[t] = kind[t] == QF_EVAL_AP ? 0 : cut[t];
  }
  if (n_queries == 0 || n_runs == 0) return QF_OK;
  if (!q_base || !docid || !score || !qrel_off || !qrel_docid || !qrel_rel || !out)
    return fail(QF_EINVAL, "qf_eval: null buffer");
  p.n_queries = n_queries;
  p.q_base = q_base;
  p.base_stride = base_stride;
  p.q_count = q_count;
  p.docid = docid;
  p.perm = perm;
  p.score = score;
  p.out_stride = out_stride;
  p.n_runs = n_runs;
  p.text_scores = text_scores != 0;
  p.qrel_off = qrel_off;
  p.qrel_docid = qrel_docid;
  p.qrel_rel = qrel_rel;
  p.n_metrics = n_metrics;
  p.out = out;
  return check(qf::eval_launch(p, (hipStream_t)stream), "qf_eval");
}

int qf_gbdt_predict(int64_t n_rows, const double* X, int32_t n_features, int32_t n_boosters,
                    const int32_t* tree_off, const int32_t* node_off, const int32_t* leaf_off,
                    const int32_t* feature, const double* threshold,
                    const int32_t* decision_type, const int32_t* left, const int32_t* right,
                    const double* leaf_value, double* out, void* stream) {
  if (n_rows < 0 || n_features <= 0 || n_boosters <= 0 || n_boosters > qf::kMaxBoosters)
    return fail(QF_EINVAL, "qf_gbdt_predict: bad sizes (n_boosters must be in [1, %d])",
                qf::kMaxBoosters);
  if (n_rows == 0) return QF_OK;
  if (!X || !tree_off || !node_off || !leaf_off || !feature || !threshold || !decision_type ||
      !left || !right || !leaf_value || !out)
    return fail(QF_EINVAL, "qf_gbdt_predict: null buffer");
  qf::GbdtParams p{n_rows, X, n_features, n_boosters, tree_off, node_off, leaf_off, feature,
                   threshold, decision_type, left, right, leaf_value, out};
  return check(qf::gbdt_predict_launch(p, (hipStream_t)stream), "qf_gbdt_predict");
}

int qf_learned_gbdt_weights(int64_t n_queries, const int64_t* micro, const double* raw_qpp,
                            const double* mm, const int64_t* list_off, int32_t norm_mode,
                            int32_t n_retrievers,
                            const int32_t* run_of_block, int32_t n_blocks, int32_t n_boosters,
                            const int32_t* tree_off, const int32_t* node_off,
                            const int32_t* leaf_off, const int32_t* feature,
                            const double* threshold, const int32_t* decision_type,
                            const int32_t* left, const int32_t* right, const double* leaf_value,
                            int32_t n_runs, const int32_t* run_to_booster, double* pred_out,
                            double* w_out, void* stream) {
  constexpr int kMaxBlocks = 256 / QF_QPP_COLS;  // the row's features staged in LDS
  if (n_queries < 0 || n_retrievers <= 0 || n_blocks <= 0 || n_blocks > kMaxBlocks ||
      n_boosters <= 0 || n_boosters > qf::kMaxBoosters || n_runs <= 0 ||
      n_runs > qf::kMaxLearnedRuns || !run_of_block || !run_to_booster)
    return fail(QF_EINVAL,
                "qf_learned_gbdt_weights: bad sizes (n_blocks in [1, %d], n_boosters in [1, %d], "
                "n_runs in [1, %d])",
                kMaxBlocks, qf::kMaxBoosters, qf::kMaxLearnedRuns);
  qf::GbdtFusedParams f{};
  f.blk.n = n_blocks;
  for (int j = 0; j < n_blocks; ++j) {
    if (run_of_block[j] < -1 || run_of_block[j] >= n_retrievers)
      return fail(QF_EINVAL, "qf_learned_gbdt_weights: run_of_block[%d] = %d out of range", j,
                  run_of_block[j]);
    f.blk.run[j] = run_of_block[j];
  }
  for (int r = 0; r < n_runs; ++r) {
    if (run_to_booster[r] < -1 || run_to_booster[r] >= n_boosters)
      return fail(QF_EINVAL, "qf_learned_gbdt_weights: run_to_booster[%d] out of range", r);
    f.lw.run_to_booster[r] = run_to_booster[r];
  }
  if (n_queries == 0) return QF_OK;
  if (!(micro || (raw_qpp && list_off && (norm_mode == QF_NORM_NONE || mm))) || !tree_off ||
      !node_off || !leaf_off || !feature || !threshold || !decision_type || !left || !right ||
      !leaf_value || !w_out)
    return fail(QF_EINVAL, "qf_learned_gbdt_weights: null buffer");
  if (!micro && norm_mode != QF_NORM_NONE && norm_mode != QF_NORM_MINMAX &&
      norm_mode != QF_NORM_ZSCORE)
    return fail(QF_EINVAL, "qf_learned_gbdt_weights: unsupported norm_mode %d", norm_mode);
  f.gbdt = qf::GbdtParams{n_queries, nullptr, n_blocks * QF_QPP_COLS, n_boosters, tree_off,
                          node_off, leaf_off, feature, threshold, decision_type, left, right,
                          leaf_value, pred_out};
  f.micro = micro;
  f.raw_qpp = raw_qpp;
  f.mm = mm;
  f.list_off = list_off;
  f.norm_mode = norm_mode;
  f.R = n_retrievers;
  f.lw.n_queries = n_queries;
  f.lw.n_boosters = n_boosters;
  f.lw.n_runs = n_runs;
  f.lw.w_out = w_out;
  return check(qf::learned_gbdt_weights_launch(f, (hipStream_t)stream), "qf_learned_gbdt_weights");
}

int qf_learned_weights(int64_t n_queries, const double* pred, int32_t n_boosters,
                       int32_t n_runs, const int32_t* run_to_booster, double* w_out,
                       void* stream) {
  if (n_queries < 0 || n_boosters <= 0 || n_boosters > qf::kMaxBoosters || n_runs <= 0 ||
      n_runs > qf::kMaxLearnedRuns || !run_to_booster)
    return fail(QF_EINVAL, "qf_learned_weights: bad sizes");
  qf::LearnedWeightParams p{};
  for (int r = 0; r < n_runs; ++r) {
    if (run_to_booster[r] < -1 || run_to_booster[r] >= n_boosters)
      return fail(QF_EINVAL, "qf_learned_weights: run_to_booster[%d] out of range", r);
    p.run_to_booster[r] = run_to_booster[r];
  }
  if (n_queries == 0) return QF_OK;
  if (!pred || !w_out) return fail(QF_EINVAL, "qf_learned_weights: null buffer");
  p.n_queries = n_queries;
  p.pred = pred;
  p.n_boosters = n_boosters;
  p.n_runs = n_runs;
  p.w_out = w_out;
  return check(qf::learned_weights_launch(p, (hipStream_t)stream), "qf_learned_weights");
}

int qf_mlp_weights(int64_t n_queries, const double* X, int32_t x_cols, const int32_t* in_col,
                   int32_t n_layers, const int32_t* widths, const float* params,
                   int32_t n_runs, const int32_t* run_to_output, double* w_out, void* stream) {
  if (n_queries < 0 || x_cols <= 0 || n_layers <= 0 || n_layers > qf::kMlpMaxLayers ||
      !widths || n_runs <= 0 || n_runs > qf::kMaxLearnedRuns || !run_to_output)
    return fail(QF_EINVAL, "qf_mlp_weights: bad sizes (1..%d layers, 1..%d runs)",
                qf::kMlpMaxLayers, qf::kMaxLearnedRuns);
  qf::MlpParams p{};
  int64_t off = 0;
  for (int l = 0; l <= n_layers; ++l) {
    if (widths[l] <= 0 || widths[l] > qf::kMlpMaxWidth)
      return fail(QF_EINVAL, "qf_mlp_weights: width[%d] = %d outside [1, %d]", l, widths[l],
                  qf::kMlpMaxWidth);
    p.width[l] = widths[l];
    if (l > 0) {
      p.w_off[l - 1] = off;
      off += (int64_t)widths[l - 1] * widths[l];
      p.b_off[l - 1] = off;
      off += widths[l];
    }
  }
  if (widths[n_layers] > qf::kMlpMaxOut)
    return fail(QF_EINVAL, "qf_mlp_weights: %d outputs exceed %d", widths[n_layers],
                qf::kMlpMaxOut);
  for (int r = 0; r < n_runs; ++r) {
    if (run_to_output[r] < -1 || run_to_output[r] >= widths[n_layers])
      return fail(QF_EINVAL, "qf_mlp_weights: run_to_output[%d] out of range", r);
    p.run_to_output[r] = run_to_output[r];
  }
  if (n_queries == 0) return QF_OK;
  if (!X || !in_col || !params || !w_out) return fail(QF_EINVAL, "qf_mlp_weights: null buffer");
  p.n_queries = n_queries;
  p.X = X;
  p.x_cols = x_cols;
  p.in_col = in_col;
  p.n_layers = n_layers;
  p.params = params;
  p.n_runs = n_runs;
  p.w_out = w_out;
  return check(qf::mlp_weights_launch(p, (hipStream_t)stream), "qf_mlp_weights");
}

int qf_synth_runs(int64_t q_begin, int64_t n_queries, int32_t n_retrievers, int32_t k,
                  uint64_t seed, double p_shared, int64_t* list_off, uint32_t* docid,
                  double* score, void* stream) {
  if (n_queries < 0 || n_retrievers <= 0 || k <= 0 || !list_off || !docid || !score)
    return fail(QF_EINVAL, "qf_synth_runs: bad arguments");
  return check(qf::synth_launch(q_begin, n_queries, n_retrievers, k, seed, p_shared, list_off,
                                docid, score, (hipStream_t)stream),
               "qf_synth_runs");
}

int qf_synth_runs_nq(int64_t q_begin, int64_t n_queries, int32_t n_retrievers, int32_t k,
                     uint64_t seed, const int64_t* qrel_off, const uint32_t* qrel_doc,
                     int64_t n_qrel_queries, int64_t* list_off, uint32_t* docid, double* score,
                     void* stream) {
  if (q_begin < 0 || n_queries < 0 || n_retrievers <= 0 || k <= 0 || k > 4096 ||
      n_qrel_queries < 0 || !list_off || (n_queries > 0 && (!docid || !score)) ||
      (n_qrel_queries > 0 && (!qrel_off || !qrel_doc)))
    return fail(QF_EINVAL, "qf_synth_runs_nq: bad arguments (1 <= k <= 4096)");
  if (2 * (int64_t)k >= 2681468)
    return fail(QF_EINVAL, "qf_synth_runs_nq: k too large for the NQ id space");
  if (seed > 0xFFFFFFFFull)  // Philox's key word: seeds differing above bit 31 would coincide
    return fail(QF_EINVAL, "qf_synth_runs_nq: seed must fit 32 bits");
  return check(qf::synth_nq_launch(q_begin, n_queries, n_retrievers, k, seed, qrel_off, qrel_doc,
                                   n_qrel_queries, list_off, docid, score, (hipStream_t)stream),
               "qf_synth_runs_nq");
}

int qf_stream_copy(void* dst, const void* src, int64_t nbytes, void* stream) {
  if (nbytes < 0 || (nbytes > 0 && (!dst || !src)) || (nbytes & 15) ||
      (((uintptr_t)dst | (uintptr_t)src) & 15))
    return fail(QF_EINVAL, "qf_stream_copy: bad arguments (16-byte aligned sizes and pointers)");
  if (nbytes == 0) return QF_OK;
  return check(qf::stream_copy_launch(dst, src, nbytes / 16, (hipStream_t)stream),
               "qf_stream_copy");
}

}  // extern "C"
