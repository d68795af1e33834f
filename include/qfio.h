/*
 * qfio.h — host-side TREC run I/O for the fusion path (libqfio.so, C++/OpenMP).
 *
 * The reference reads runs with pandas (load_runs, src/fusion.py:46-76:
 * read_csv(sep=r"\s+", names=[qid, iter, docno, rank, score, runid], qid and
 * docno as str)) and writes fused runs with a Python loop (write_runfile,
 * src/fusion.py:480-492).  These entry points do the same work natively and
 * produce the packed layout of include/qppfuse.h directly.  Host pointers only.
 */
#ifndef QFIO_H
#define QFIO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QFIO_OK     0
#define QFIO_EINVAL 1
#define QFIO_ENOENT 2 /* a file cannot be opened (FileNotFoundError)  */
#define QFIO_EIO    3
#define QFIO_EPARSE 4 /* a line is not "qid Q0 docno rank score tag" */
#define QFIO_EPYTHON 5 /* the file needs the reference's own Python reading (see
                          qfio_read_score_lists); nothing is returned */

typedef struct qfio_runset qfio_runset;

const char* qfio_last_error(void);

/*
 * Parse n_files run files (one run each, in the given order = the runs dict
 * order) with n_threads threads (<= 0: OpenMP default).  Queries are the
 * sorted distinct qids, docnos are interned in byte (= Python str) order; the
 * CSR list (q, r) holds file r's rows of query q in file order.
 */
int qfio_load_runs(const char* const* paths, int32_t n_files, int32_t n_threads,
                   qfio_runset** out);
/* sizes[8]: n_queries, n_docnos, n_entries, qid bytes, docno bytes,
 * flags (bit 0 micro_ok: every score is an exact 6-decimal number; bit 1: every
 * rank equals position + 1; bit 2: every list is score-descending with strictly
 * rising ranks), n_iter | n_tag << 32,
 * iter bytes | tag bytes << 32 */
void qfio_runset_sizes(const qfio_runset* rs, int64_t* sizes);
/* CSR: list_off[Q*R+1], docid[E], score[E], micro[E] (nullable; only if
 * micro_ok), rank[E] (file rank column) */
int qfio_runset_csr(const qfio_runset* rs, int64_t* list_off, uint32_t* docid, double* score,
                    int32_t* micro, int64_t* rank);
/* interned strings: offsets [n+1] + concatenated bytes, for qids, docnos, the
 * iter column and the tag column */
int qfio_runset_strings(const qfio_runset* rs, int64_t* qid_off, char* qid_chars,
                        int64_t* docno_off, char* docno_chars, int64_t* iter_off,
                        char* iter_chars, int64_t* tag_off, char* tag_chars);
/* strings i = chars[off[i], off[i+1]) of a table, each followed by '\n', into
 * out (off[n] + n bytes): one decode + split gives Python str objects (no field
 * of a whitespace-separated run file contains '\n') */
int qfio_join_lines(const int64_t* off, const char* chars, int64_t n, char* out);
/* rows of every file in file order (the DataFrames load_runs returns):
 * file_off[R+1], codes into qids / docnos / iters / tags, rank, score */
int qfio_runset_rows(const qfio_runset* rs, int64_t* file_off, uint32_t* qid, uint32_t* docid,
                     uint32_t* iter, uint32_t* tag, int64_t* rank, double* score);
/* the same columns without copies: pointers [12] into the run set (valid until
 * qfio_runset_free) to list_off, docid, score, micro (NULL unless micro_ok),
 * rank, file_off, and the row codes / rank / score of qfio_runset_rows */
void qfio_runset_views(const qfio_runset* rs, const void** ptrs);
/* after qfio_runset_strings: release the string views and unmap the files (the
 * columns stay); qfio_runset_sizes / _strings must not be called after it */
void qfio_runset_drop_text(qfio_runset* rs);
void qfio_runset_free(qfio_runset* rs);
/* per-row strings of a column given as codes into a table (offsets [m+1] +
 * bytes): out_off[n+1] (int64, Arrow large_string offsets) always, the bytes
 * into out_chars when it is not NULL (size: the return value of a first call
 * with out_chars = NULL).  Returns the byte count, -1 on bad arguments. */
int64_t qfio_gather_strings(const int64_t* tab_off, const char* tab_chars, const uint32_t* codes,
                            int64_t n, int64_t* out_off, char* out_chars);
/* the bytes of a column whose out_off[n+1] a first qfio_gather_strings call
 * (out_chars = NULL, same codes) has filled: one pass instead of a second
 * qfio_gather_strings.  Returns 0, -1 on bad arguments. */
int qfio_gather_chars(const int64_t* tab_off, const char* tab_chars, const uint32_t* codes,
                      int64_t n, const int64_t* out_off, char* out_chars);
/* Arrow offsets of n repeats of one len-byte string: out_off[i] = i * len, i <= n
 * (a column of one value: iter "Q0", a run's tag). */
void qfio_repeat_offsets(int64_t len, int64_t n, int64_t* out_off);
/* A 64-bit content digest of nbytes at data, hashed over the threads (the pack
 * cache's fingerprint of the numeric columns load_runs returns; not cryptographic). */
uint64_t qfio_hash_bytes(const void* data, int64_t nbytes);

/* Python's f"{x:.6f}" of x into out (>= 400 bytes); returns the length. */
size_t qfio_format_score(double x, char* out);

/*
 * write_runfile for one fused run (qf_fuse outputs copied to the host):
 * queries order[0..n_out) (indices into qbase / counts / qid strings), for each
 * its counts[q] documents u = qbase[q] + perm[qbase[q] + k] with rank k + 1:
 * docno union_docid[u], score fused[u] (qf_fuse's layout: scores in first-seen
 * order, perm ranks them); one line "qid Q0 docno rank score tag".
 */
int qfio_write_run(const char* path, int64_t n_out, const int64_t* order, const int64_t* qbase,
                   const int32_t* counts, const uint32_t* union_docid, const uint16_t* perm,
                   const double* fused, const int64_t* qid_off, const char* qid_chars,
                   const int64_t* docno_off, const char* docno_chars, const char* tag,
                   int32_t n_threads);
/* The same for qf_fuse_wide's uint32 perm. */
int qfio_write_run32(const char* path, int64_t n_out, const int64_t* order, const int64_t* qbase,
                     const int32_t* counts, const uint32_t* union_docid, const uint32_t* perm,
                     const double* fused, const int64_t* qid_off, const char* qid_chars,
                     const int64_t* docno_off, const char* docno_chars, const char* tag,
                     int32_t n_threads);

/*
 * compute_qpp_for_res_file's read of a RAW run file (src/qpp.py:292-305): every
 * line with >= 5 whitespace-separated fields adds float(field 5) to its qid's
 * list in file order; qids in first-appearance order; each list sorted descending
 * (stable: -0.0 / 0.0 keep file order, as sorted(reverse=True)) and sliced
 * [:top_k] with Python's slice semantics (negative top_k drops from the end).
 * QFIO_EPARSE: a fifth field float() rejects (message = Python's ValueError text).
 * QFIO_EPYTHON: the file holds something only Python's reading decides exactly
 * (bytes >= 0x80 or 0x1c-0x1f, a lone '\r', digit underscores, a NaN score).
 */
typedef struct qfio_scorelists qfio_scorelists;
int qfio_read_score_lists(const char* path, int32_t top_k, int32_t n_threads,
                          qfio_scorelists** out);
/* sizes[4]: n_queries, kept scores, qid bytes, rows read (lines with >= 5 fields) */
void qfio_scorelists_sizes(const qfio_scorelists* s, int64_t* sizes);
/* qid_off[Q+1] + qid_chars (first-appearance order), list_off[Q+1], scores */
int qfio_scorelists_get(const qfio_scorelists* s, int64_t* qid_off, char* qid_chars,
                        int64_t* list_off, double* scores);
void qfio_scorelists_free(qfio_scorelists* s);

#ifdef __cplusplus
}
#endif
#endif /* QFIO_H */
