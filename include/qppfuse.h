/*
 * qppfuse.h — C-ABI of the MI355X-native fusion + QPP engine (libqppfuse.so).
 *
 * This is the drop-in boundary for the hot path of PoisedDok/QPP-Fusion-RAG:
 *   src/fusion.py   (combsum/combmnz/rrf :170-230, weighted_* :237-380)
 *   src/qpp.py      (compute_qpp_for_res_file :245-337, _normalize_qpp :340-374)
 *   src/qpp/java/qpp/QPPBridge.java (computeQPPScores :134-191, predictors :202-453)
 *   src/retrievers/base.py (normalize_scores :60-73)
 * The reference has no FFI of its own (Python + a JVM subprocess speaking JSON,
 * src/qpp.py:140-147); every entry point below replaces one of those functions and
 * names it.  The Python mirror of the reference API (qppfuse.fusion / qppfuse.qpp)
 * binds these symbols with ctypes — see INTEGRATION.md.
 *
 * Conventions
 *  - Every pointer argument is a DEVICE pointer (HBM) unless stated otherwise;
 *    the library never allocates or frees caller memory.
 *  - `stream` is a hipStream_t passed as void*; all work is stream-ordered and
 *    asynchronous.  Functions are re-entrant; they use the current HIP device.
 *  - Return value: QF_OK or an error code; qf_last_error() (thread-local) says why.
 *  - Run lists are stored query-major in CSR form: list (q, r) of query q and
 *    retriever r occupies entries [list_off[q*R + r], list_off[q*R + r + 1]).
 */
#ifndef QPPFUSE_H
#define QPPFUSE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------- */
#define QF_OK       0
#define QF_EINVAL   1 /* bad argument (null pointer, bad size, unknown method)   */
#define QF_ETOOBIG  2 /* a query has more entries than the fusion kernel holds   */
#define QF_EHIP     3 /* HIP runtime error (launch / device)                     */

/* Per-query status written to union_count[q] by qf_fuse when it is negative. */
#define QF_QSTATUS_TOOBIG    (-1) /* query exceeds qf_max_entries_per_query()   */
#define QF_QSTATUS_UNSORTED  (-2) /* a list is not sorted by score, descending  */
#define QF_QSTATUS_RANKORDER (-3) /* rank column not non-decreasing in a list   */
#define QF_QSTATUS_BADDOC    (-4) /* docid 0xFFFFFFFF (reserved) seen           */
#define QF_QSTATUS_DUPDOC    (-5) /* a docid repeats inside one (q, r) list     */

/* ---- fusion methods (bit mask; output slot m = m-th set bit, ascending) -- */
#define QF_COMBSUM  (1 << 0) /* ranx fuse(method="sum")   src/fusion.py:170-186 */
#define QF_COMBMNZ  (1 << 1) /* ranx fuse(method="mnz")   src/fusion.py:189-205 */
#define QF_RRF      (1 << 2) /* ranx fuse(method="rrf")   src/fusion.py:208-230 */
#define QF_WCOMBSUM (1 << 3) /* weighted_combsum          src/fusion.py:237-281 */
#define QF_WCOMBMNZ (1 << 4) /* weighted_combmnz          src/fusion.py:284-330 */
#define QF_WRRF     (1 << 5) /* weighted_rrf              src/fusion.py:333-380 */
#define QF_LEARNED  (1 << 6) /* learned_fusion's sum      src/fusion.py:436-446:
                                sum of score * w per (qid, docno) in pandas'
                                groupby-sum (Kahan) order; ties by docno.  Takes
                                its weights (qf_learned_weights) in `weights`, so
                                it cannot share a call with the W-* methods. */
#define QF_PROBFUSE (1 << 7) /* probFuse (ProbFuse.py:136-187 build_probfuse_run):
                                sum over runs of P_r[seg - 1] / seg, seg =
                                ceil(rank * x / L) clipped to [1, x], rank = the
                                file rank column; only via qf_fuse_probfuse */
#define QF_WRRF_MUL (1 << 8) /* QPPrrf_argmax.py:53-76 build_rrf_run: sum over runs
                                of w_r * (1 / (k + rank)), file rank column, rows
                                in file order (weights 1.0 = its plain RRF) */
#define QF_ALL_METHODS 0x3F  /* the six fusions of config.fusion.methods */

/* ---- score column encodings --------------------------------------------- */
#define QF_SCORE_F64   0 /* double                                              */
#define QF_SCORE_MICRO 1 /* int32 micro-units, value = m / 1e6 (exact %.6f text) */

/* ---- QPP normalisation modes (src/qpp.py:340-374) ----------------------- */
#define QF_NORM_NONE   0
#define QF_NORM_MINMAX 1
#define QF_NORM_ZSCORE 2

#define QF_QPP_COLS 13 /* Java column order: nqc smv wig SigmaMax SigmaX RSD UEF
                          MaxIDF avgidf cumnqc snqc dense-qpp dense-qpp-m
                          (QPPBridge.java:148-188, config/defaults.yaml:164-177) */

const char* qf_version(void);
const char* qf_last_error(void);
/* Largest Σ_r |list(q,r)| one query may have for qf_fuse (65,535: perm is
 * uint16) and for the *_wide entry points (16,777,215: perm is uint32). */
int qf_max_entries_per_query(void);
int qf_max_entries_per_query_wide(void);

/*
 * Per-query min-max normalisation of every list (BaseRetriever.normalize_scores,
 * src/retrievers/base.py:60-73): (s - min) / (max - min), range -> 1.0 when
 * max == min.  out_norm (nullable) gets the double; out_micro (nullable) gets
 * the value rounded exactly as Python's f"{x:.6f}" (scripts/02_retrieve.py:80),
 * in micro-units — i.e. exactly what the .norm.res text holds.
 */
int qf_minmax_per_query(const double* score, const int64_t* list_off, int64_t n_lists,
                        double* out_norm, int32_t* out_micro, void* stream);

/*
 * Raw QPP predictors, one row of QF_QPP_COLS doubles per list
 * (QPPBridge.computeQPPScores, QPPBridge.java:134-191, after the driver's
 * sort-desc + [:top_k] truncation, src/qpp.py:304-305).  Lists must be sorted
 * by score, descending.  Scores are rounded to float32 as Java's
 * JsonElement.getAsFloat() does (QPPBridge.java:67-70), then the first
 * k = min(50, n) are used.  num_terms[q] = max(1, |lower(text).split("\\s+")|),
 * text_feat[2q], text_feat[2q+1] = MaxIDF / avgidf proxies (host string work,
 * QPPBridge.java:368-393).  Empty lists get an all-zero row (Java returns an
 * empty map; src/qpp.py:321 maps missing names to 0.0).
 */
int qf_qpp_raw(const double* score, const int64_t* list_off, int64_t n_queries,
               int32_t n_retrievers, int32_t top_k, const int32_t* num_terms,
               const double* text_feat, double* raw_out, void* stream);

/*
 * Column minima / maxima of the raw predictors over the queries of each
 * retriever that have a non-empty list (src/qpp.py:347-358).  mm_out holds
 * 2*R*13 doubles: [0, R*13) = min, [R*13, 2*R*13) = -max, so that a single
 * element-wise MIN all-reduce (RCCL) combines query shards.
 */
int qf_qpp_colminmax(const double* raw, const int64_t* list_off, int64_t n_queries,
                     int32_t n_retrievers, double* mm_out, void* stream);

/*
 * qf_minmax_per_query (micro-units and / or normalised scores of the n_queries *
 * n_retrievers lists) and qf_qpp_colminmax (of raw_qpp into mm_out) in ONE launch —
 * the two independent reductions of an unsharded step; the same bits as the two
 * calls.  (A sharded step keeps them apart: the column extremes go through the MIN
 * all-reduce while the min-max kernel runs.)
 */
int qf_minmax_colminmax(const double* score, const int64_t* list_off, int64_t n_queries,
                        int32_t n_retrievers, double* out_norm, int32_t* out_micro,
                        const double* raw_qpp, double* mm_out, void* stream);

/*
 * zscore statistics (src/qpp.py:358-359): per (retriever, column) numpy's
 * arr.mean() and the scale arr.std() (population; 1.0 when not > 0) over the
 * queries with a non-empty list, in query order.  Bit-identical to numpy: its
 * float64 sum is reproduced exactly (0.0 + pairwise sums of 8192-element
 * chunks; pairwise = numpy's fixed recursion with 8 accumulators below 128).
 * st_out holds 2*R*13 doubles: [0, R*13) = mean, [R*13, 2*R*13) = scale.
 * Queries are not shardable for this (the sum's tree depends on positions):
 * one device sees every query.
 */
int qf_qpp_colmeanstd(const double* raw, const int64_t* list_off, int64_t n_queries,
                      int32_t n_retrievers, double* st_out, void* stream);

/*
 * Normalise raw predictors (src/qpp.py:362-372) — mode QF_NORM_MINMAX with
 * mm from qf_qpp_colminmax, QF_NORM_ZSCORE with mm from qf_qpp_colmeanstd,
 * QF_NORM_NONE without — and round each value
 * as the .qpp writer's f"{s:.6f}" does (src/qpp.py:333): micro_out (nullable,
 * int64 micro-units) and norm_out (nullable, the unrounded double).  Then, if
 * w_out is non-null, the fusion weight of every (q, r) as
 * get_qpp_weight (src/fusion.py:116-158) reads it back from the .qpp text:
 * column qpp_index, or the mean of the 13 columns when qpp_index == -1.
 */
int qf_qpp_normalize(const double* raw, const double* mm, const int64_t* list_off,
                     int64_t n_queries, int32_t n_retrievers, int32_t mode,
                     int32_t qpp_index, double* norm_out, int64_t* micro_out,
                     double* w_out, void* stream);

/*
 * Learned fusion's feature matrix on device: X[q, j*13 + c] = the "%.6f" value
 * of normalised predictor c of run run_of_block[j] (micro_out of
 * qf_qpp_normalize, / 1e6 exactly as the .qpp text reads back), i.e. the
 * X[Q, 13 * n_model_retrievers] learned_fusion builds from qpp_data
 * (src/fusion.py:415-427; src/data_utils.py:262-293).  run_of_block: host array
 * of n_blocks (<= 32) run indices, -1 = a retriever the batch lacks (zeros).
 */
int qf_qpp_features(const int64_t* micro, int64_t n_queries, int32_t n_retrievers,
                    const int32_t* run_of_block, int32_t n_blocks, double* X, void* stream);

/*
 * Multi-method rank fusion of every query: a join kernel (one workgroup per
 * query: LDS hash join over docids, contribution groups in first-seen order,
 * the ordered sums of every requested method) and a sort kernel (one workgroup
 * per (query, method): stable LDS bucket sort by fused score, which writes the
 * rank order as perm).
 * Queries of 10,241 .. qf_max_entries_per_query() (65,535) entries take a third
 * kernel (the same join in a global workspace + the bucket sort over the
 * workspace), launched only when max_entries > 10,240 (or n_retrievers > 16),
 * with a workspace allocated and freed stream-ordered (hipMallocAsync /
 * hipFreeAsync on `stream`) — the one internal allocation; qf_fuse_ws below takes
 * a caller-owned workspace instead.  Larger queries (up
 * to qf_max_entries_per_query_wide()) need qf_fuse_wide: u can exceed 65,535.
 * max_entries must bound every query's entry count (larger queries report
 * QF_QSTATUS_TOOBIG).  n_retrievers <= 32; with more than 16 every query takes
 * the workspace kernel (its retriever masks are 32-bit, the LDS join's 16-bit).
 *
 * Inputs (device): list_off[Q*R+1] (int64), docid[E] (uint32, interned
 * docnos, 0xFFFFFFFF reserved), score[E] (score_kind), rank[E] (nullable
 * int32 file rank column for W-RRF, src/fusion.py:372-374; NULL = position+1),
 * weights[Q*R] (nullable unless a weighted method is requested).
 * Preconditions per list: scores non-increasing; no docid repeated.
 *
 * Outputs (device), query q owns slots [list_off[q*R], list_off[q*R+R]):
 *   union_docid  — the query's distinct docids in first-seen order
 *                  (retriever order, then list position), u = 0..U_q-1
 *   union_count[q] = U_q (or a negative QF_QSTATUS_* code)
 *   for the m-th requested method (ascending bit order), at offset m*out_stride:
 *     fused[... + u] — document u's fused score (double), first-seen order
 *     perm[... + i]  — the u of rank i: scores descending, ties in first-seen
 *                      order (Python's stable sort, src/fusion.py:475,488)
 *   so rank i of query q is union_docid[b + perm[b + i]] with score
 *   fused[b + perm[b + i]], b = list_off[q*R] (+ m*out_stride for perm / fused).
 *   The scores are written once, by the join; the sort writes only perm.
 *   Slots [b + U_q, b + N_q) of a query's fused / perm rows (N_q its entries) are
 *   scratch: the join may leave the sort's key constants there.
 */
int qf_fuse(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
            const uint32_t* docid, const void* score, int32_t score_kind,
            const int32_t* rank, const double* weights, int32_t methods, int32_t rrf_k,
            int32_t max_entries, uint32_t* union_docid, int32_t* union_count,
            uint16_t* perm, double* fused, int64_t out_stride, void* stream);

/*
 * qf_fuse with the W-* weights taken from the QPP predictors themselves: the raw
 * predictors qpp_raw [n_queries * n_retrievers][13] and their column statistics
 * qpp_stats (qf_qpp_colminmax's [min, -max] for QF_NORM_MINMAX, qf_qpp_colmeanstd's
 * [mean, scale] for QF_NORM_ZSCORE; unused for QF_NORM_NONE), column qpp_index
 * (-1: the mean of the 13) — the weights qf_qpp_normalize's w_out would hold, bit
 * for bit, computed inside the fusion (src/qpp.py:356-372 + the .qpp round trip of
 * get_qpp_weight, src/fusion.py:116-158): one launch fewer per batch.  Not with
 * QF_LEARNED.  Meant for one column: qpp_index -1 puts 13 normalisations per list
 * on the start of every query's workgroup (C4: slower than qf_qpp_normalize +
 * qf_fuse).
 */
int qf_fuse_qpp(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
                const uint32_t* docid, const void* score, int32_t score_kind, const int32_t* rank,
                const double* qpp_raw, const double* qpp_stats, int32_t qpp_mode,
                int32_t qpp_index, int32_t methods, int32_t rrf_k, int32_t max_entries,
                uint32_t* union_docid, int32_t* union_count, uint16_t* perm, double* fused,
                int64_t out_stride, void* stream);

/*
 * qf_fuse_qpp + the .qpp file's values: the join also writes qpp_micro_out[(q*R +
 * r)*13 + c] = the "%.6f" micro-units of normalised predictor c of list (q, r) —
 * qf_qpp_normalize's micro_out, bit for bit (src/qpp.py:324-334, 356-372) — for
 * every column, so one fusion launch produces both the fused runs and the whole
 * .qpp table the metric's "13 QPP" names.  n_retrievers <= 16.
 */
int qf_fuse_qpp_micro(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
                      const uint32_t* docid, const void* score, int32_t score_kind,
                      const int32_t* rank, const double* qpp_raw, const double* qpp_stats,
                      int32_t qpp_mode, int32_t qpp_index, int32_t methods, int32_t rrf_k,
                      int32_t max_entries, uint32_t* union_docid, int32_t* union_count,
                      uint16_t* perm, double* fused, int64_t out_stride, int64_t* qpp_micro_out,
                      void* stream);

/*
 * The explicit workspace of qf_fuse (the library allocates only in
 * an explicit workspace).  qf_fuse_workspace_bytes: the bytes a call with these
 * sizes would allocate stream-ordered for its workspace kernel (queries above
 * 10,240 entries, or more than 16 runs); 0 when the call needs none.
 * qf_fuse_ws = qf_fuse (wide = 0: uint16 perm) or qf_fuse_wide (wide = 1: uint32
 * perm) with a caller-owned device workspace: ws = NULL keeps the stream-ordered
 * allocation; otherwise ws must be 256-byte aligned (its workgroup shares hold
 * u32 atomicCAS targets and u64 sort words; a misaligned ws fails with
 * QF_EINVAL) and ws_bytes must hold at least one workgroup's share (the call
 * fails with QF_EINVAL naming it), and a workspace smaller than
 * qf_fuse_workspace_bytes runs the workspace kernel with fewer workgroups (same
 * results).  The workspace needs no initialisation and may be reused by the next
 * call on the same stream; the library never frees it.
 */
int64_t qf_fuse_workspace_bytes(int64_t n_queries, int32_t n_retrievers, int32_t max_entries,
                                int32_t methods, int32_t wide);
int qf_fuse_ws(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
               const uint32_t* docid, const void* score, int32_t score_kind, const int32_t* rank,
               const double* weights, int32_t methods, int32_t rrf_k, int32_t max_entries,
               uint32_t* union_docid, int32_t* union_count, void* perm, int32_t wide,
               double* fused, int64_t out_stride, void* ws, size_t ws_bytes, void* stream);

/*
 * qf_fuse, qf_fuse_probfuse, qf_fuse_learned_f32 and qf_fused_topk with a uint32
 * perm [M][E]: every query up to qf_max_entries_per_query_wide() entries (its
 * union's u may exceed 65,535).  Same outputs, same order, same errors; one call
 * is all-uint32 (the small queries' perm too).  The reference has no per-query
 * size limit (src/fusion.py:264-279 builds Python dicts): these lift qf_fuse's.
 */
int qf_fuse_wide(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
                 const uint32_t* docid, const void* score, int32_t score_kind,
                 const int32_t* rank, const double* weights, int32_t methods, int32_t rrf_k,
                 int32_t max_entries, uint32_t* union_docid, int32_t* union_count,
                 uint32_t* perm, double* fused, int64_t out_stride, void* stream);
int qf_fuse_probfuse_wide(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
                          const uint32_t* docid, const void* score, int32_t score_kind,
                          const int32_t* rank, const double* weights, int32_t methods,
                          int32_t rrf_k, const double* seg_prob, int32_t n_segments,
                          int32_t seg_len, int32_t max_entries, uint32_t* union_docid,
                          int32_t* union_count, uint32_t* perm, double* fused,
                          int64_t out_stride, void* stream);
int qf_fuse_learned_f32_wide(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
                             const uint32_t* docid, const void* score, int32_t score_kind,
                             const double* weights, uint32_t f32_runs, int32_t max_entries,
                             uint32_t* union_docid, int32_t* union_count, uint32_t* perm,
                             double* fused, int64_t out_stride, void* stream);
int qf_fused_topk_wide(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
                       const int32_t* union_count, const uint32_t* union_docid,
                       const uint32_t* perm, const double* fused, int64_t out_stride,
                       int32_t n_methods, int32_t k, uint32_t* out_docid, double* out_score,
                       void* stream);

/*
 * qf_fuse with the ProbFuse segment table (ProbFuse.py:136-187): `methods` may
 * add QF_PROBFUSE to the qf_fuse methods; seg_prob[r * n_segments + k - 1] is
 * P_k of run r (train_probfuse, ProbFuse.py:92-133; zeros for a run the model
 * does not know), n_segments = x, seg_len = L.  Other arguments as qf_fuse.
 */
int qf_fuse_probfuse(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
                     const uint32_t* docid, const void* score, int32_t score_kind,
                     const int32_t* rank, const double* weights, int32_t methods,
                     int32_t rrf_k, const double* seg_prob, int32_t n_segments,
                     int32_t seg_len, int32_t max_entries, uint32_t* union_docid,
                     int32_t* union_count, uint16_t* perm, double* fused, int64_t out_stride,
                     void* stream);

/*
 * Fused top-k of every (query, method slot) from qf_fuse's outputs, packed for
 * the multi-GPU gather of the final fused lists (qppfuse.dist.gather_fused_topk):
 * out_docid / out_score[(q * n_methods + m) * k + i] = rank i (< min(k, U_q)) of
 * method slot m — docid union_docid[base + perm[...]], its fused score; the rest
 * of each row is docid 0xFFFFFFFF / score NaN.  base = list_off[q * R].
 */
int qf_fused_topk(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
                  const int32_t* union_count, const uint32_t* union_docid, const uint16_t* perm,
                  const double* fused, int64_t out_stride, int32_t n_methods, int32_t k,
                  uint32_t* out_docid, double* out_score, void* stream);

/*
 * LightGBM inference for learned fusion (src/fusion.py:415-429 ->
 * MultiOutputLGBM / PerRetrieverLGBM .predict, src/models/lightgbm_models.py):
 * out[row*n_boosters + b] = raw prediction of booster b on X[row*n_features ..]
 * (its first best_iteration trees).  The model is flat arrays (qppfuse/lgbm.py
 * pack_model): trees of booster b = [tree_off[b], tree_off[b+1]); internal nodes
 * of tree t = [node_off[t], node_off[t+1]) with feature / threshold /
 * decision_type (LightGBM bits: 2 = default left, (d >> 2) & 3 = missing type)
 * / left / right (child >= 0: node, < 0: leaf ~child); leaves of tree t =
 * leaf_value[leaf_off[t] ..].  Numerical splits only.  All pointers device.
 */
int qf_gbdt_predict(int64_t n_rows, const double* X, int32_t n_features, int32_t n_boosters,
                    const int32_t* tree_off, const int32_t* node_off, const int32_t* leaf_off,
                    const int32_t* feature, const double* threshold,
                    const int32_t* decision_type, const int32_t* left, const int32_t* right,
                    const double* leaf_value, double* out, void* stream);

/*
 * Learned weights (src/models/base.py:120-125 _normalize_weights, then
 * src/fusion.py:431-440): per query clip the n_boosters predictions at 0,
 * divide by their numpy row sum (1 when 0); run r gets the weight of booster
 * run_to_booster[r] (HOST array, n_runs <= 32), or 1/n_boosters when it is -1
 * (a run the model does not know).  w_out[q*n_runs + r] feeds qf_fuse(QF_LEARNED).
 */
int qf_learned_weights(int64_t n_queries, const double* pred, int32_t n_boosters,
                       int32_t n_runs, const int32_t* run_to_booster, double* w_out,
                       void* stream);

/*
 * qf_qpp_features + qf_gbdt_predict + qf_learned_weights in ONE launch (the step
 * src/fusion.py:415-440 takes from the .qpp values to the run weights): row q's
 * features are the QPP micro-units laid out as qf_qpp_features lays them out
 * (run_of_block: HOST array, n_blocks <= 19 so the 13 * n_blocks features fit the
 * kernel's LDS row) — read from `micro`, or, when micro is NULL, normalised on the
 * fly from raw_qpp with the column statistics mm (norm_mode QF_NORM_*; list_off
 * marks absent lists) exactly as qf_qpp_normalize would — the model walked as
 * qf_gbdt_predict does, and w_out filled as qf_learned_weights does: the same bits
 * as the separate calls.  pred_out (nullable): the raw predictions [n_queries][B].
 */
int qf_learned_gbdt_weights(int64_t n_queries, const int64_t* micro, const double* raw_qpp,
                            const double* mm, const int64_t* list_off, int32_t norm_mode,
                            int32_t n_retrievers,
                            const int32_t* run_of_block, int32_t n_blocks, int32_t n_boosters,
                            const int32_t* tree_off, const int32_t* node_off,
                            const int32_t* leaf_off, const int32_t* feature,
                            const double* threshold, const int32_t* decision_type,
                            const int32_t* left, const int32_t* right, const double* leaf_value,
                            int32_t n_runs, const int32_t* run_to_booster, double* pred_out,
                            double* w_out, void* stream);

/*
 * FusionMLP learned fusion (src/models/mlp_model.py:254-274 predict, called by
 * src/fusion.py:429 -> replaces `pred_weights = model.predict(X)` for the MLP model
 * and the weights' lookup at :440).  Model input i is X[q*x_cols + in_col[i]]
 * (in_col: DEVICE int32 [widths[0]], _filter_features' column map), rounded to
 * float32.  n_layers Linear layers, widths[0..n_layers] (HOST array, each <= 512,
 * outputs <= 32), ReLU between them; params (DEVICE float32) holds layer l's
 * W [widths[l+1]][widths[l]] then b [widths[l+1]], layer after layer.  The output
 * goes through softmax and _normalize_weights (src/models/base.py:120-125) in
 * float32; w_out[q*n_runs + r] = weight of output run_to_output[r] (HOST array), or
 * 1/widths[n_layers] for -1.  The float32 operation order is fixed (see
 * csrc/qf_learn.hip); torch's CPU/MPS kernels round differently by a few ulps.
 */
int qf_mlp_weights(int64_t n_queries, const double* X, int32_t x_cols, const int32_t* in_col,
                   int32_t n_layers, const int32_t* widths, const float* params,
                   int32_t n_runs, const int32_t* run_to_output, double* w_out, void* stream);

/*
 * qf_fuse(QF_LEARNED) with FusionMLP's float32 weights (src/fusion.py:436-441
 * under numpy 2: row["score"] * np.float32 is a float32 product).  Bit r of
 * f32_runs: run r's weight is a float32 model output (its products round to
 * float32); runs without the bit (unknown to the model: 1.0 / n_retrievers) take
 * float64 products.  With every run's bit set the groupby sum is float32 Kahan
 * (pandas' float32 column), otherwise float64 Kahan.  Outputs as qf_fuse, one
 * method (QF_LEARNED).
 */
int qf_fuse_learned_f32(int64_t n_queries, int32_t n_retrievers, const int64_t* list_off,
                        const uint32_t* docid, const void* score, int32_t score_kind,
                        const double* weights, uint32_t f32_runs, int32_t max_entries,
                        uint32_t* union_docid, int32_t* union_count, uint16_t* perm,
                        double* fused, int64_t out_stride, void* stream);

/* ---- IR evaluation (trec_eval semantics, as ir_measures computes them) ---- */
#define QF_EVAL_NDCG 0 /* nDCG@k   */
#define QF_EVAL_RR   1 /* RR@k     */
#define QF_EVAL_R    2 /* R@k      */
#define QF_EVAL_P    3 /* P@k      */
#define QF_EVAL_AP   4 /* AP (cut ignored) */
#define QF_EVAL_MAX_METRICS 16
#define QF_EVAL_MAX_QRELS 256 /* judged documents per query */

/*
 * Evaluation of ranked runs against qrels — the metrics scripts/06_eval_fusion.py
 * gets from ir_measures (src/evaluation/ir_evaluator.py:51-86, metric list
 * config/defaults.yaml:224-234) on the fused .res files.  Documents are ranked by
 * score descending, ties by docno descending (trec_eval), which is docid
 * descending when docids are interned in docno string order.  text_scores != 0
 * takes every score as the "%.6f" text write_runfile prints (src/fusion.py:491)
 * and 06_eval_fusion reads back; 0 takes the doubles as they are.
 *
 * Run m (0..n_runs-1), query q: its list is sorted by score descending and holds
 * n_q = q_count[q] (or, q_count NULL, q_base[(q+1)*base_stride] - b) entries at
 * b = q_base[q*base_stride]:  score[m*out_stride + b + i], and docid
 * docid[b + perm[m*out_stride + b + i]] when perm is non-NULL (qf_fuse's
 * outputs: q_base = list_off, base_stride = R, q_count = union_count, docid =
 * union_docid), else docid[m*out_stride + b + i].
 * Qrels (device): qrel_off[Q+1] (int64), qrel_docid (uint32, ascending inside a
 * query), qrel_rel (int32); at most max_qrels <= QF_EVAL_MAX_QRELS per query.
 * Metrics (HOST arrays): kind[t] (QF_EVAL_*), cut[t] (k >= 1; ignored for AP).
 * out[(m*Q + q)*n_metrics + t] (device double): the value, or NaN when the query
 * has no entries or no qrels (trec_eval does not evaluate it).
 */
int qf_eval(int64_t n_queries, const int64_t* q_base, int32_t base_stride,
            const int32_t* q_count, const uint32_t* docid, const uint16_t* perm,
            const double* score, int64_t out_stride, int32_t n_runs, int32_t text_scores,
            const int64_t* qrel_off, const uint32_t* qrel_docid, const int32_t* qrel_rel,
            int32_t max_qrels, int32_t n_metrics, const int32_t* kind, const int32_t* cut,
            double* out, void* stream);

/*
 * Benchmark / test support: generate Q*R synthetic lists of K entries
 * (docid, raw score sorted descending) on device, deterministic in seed.
 * list_off[Q*R+1] is written too.  See DESIGN.md "Synthetic runs".
 */
int qf_synth_runs(int64_t q_begin, int64_t n_queries, int32_t n_retrievers, int32_t k,
                  uint64_t seed, double p_shared, int64_t* list_off, uint32_t* docid,
                  double* score, void* stream);

/*
 * Benchmark / test support: the synthetic runs SURVEY.md §8(d) specifies — per
 * query and retriever (BGE, BM25, BM25_MonoT5, BM25_TCT, Splade order) K distinct
 * docids, each with probability 0.5 from the query's shared pool of 2K NQ corpus ids
 * else from the rest of the 2,681,468; raw scores sorted descending + 1e-6 * (K - 1 -
 * rank): Gamma(2, 6) + 5 (BM25, Splade), 0.5 + 0.4 Beta(5, 2) (BGE, BM25_TCT),
 * ln Beta(5, 2) - 0.001 (BM25_MonoT5, negative); the judged documents of qrel query q mod
 * n_qrel_queries (device CSR qrel_off[n+1] / qrel_doc: corpus ids) planted with
 * probability {0.9, 0.5, 0.9, 0.8, 0.9} at Geometric(0.15) ranks.  Counter-based
 * (Philox4x32-10 keyed by seed, a 32-bit key word: seed > 0xFFFFFFFF fails with
 * QF_EINVAL): any query range regenerates independently; oracle/synth_oracle.c
 * regenerates it bit for bit.  1 <= k <= 4096.
 */
int qf_synth_runs_nq(int64_t q_begin, int64_t n_queries, int32_t n_retrievers, int32_t k,
                     uint64_t seed, const int64_t* qrel_off, const uint32_t* qrel_doc,
                     int64_t n_qrel_queries, int64_t* list_off, uint32_t* docid, double* score,
                     void* stream);

/*
 * Measurement support (bench.py's roofline): a device-to-device streaming copy of
 * nbytes (a multiple of 16; 16-byte aligned pointers), 16 bytes per lane, one
 * non-temporal access per thread over a one-shot grid (the fastest shape measured).  Its rate (2 * nbytes / time) is the practical HBM
 * ceiling the roofline object reports next to the 8 TB/s spec peak.  No
 * counterpart in the reference.
 */
int qf_stream_copy(void* dst, const void* src, int64_t nbytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* QPPFUSE_H */
