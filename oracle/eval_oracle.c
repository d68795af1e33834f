/*
 * eval_oracle.c — TEST INFRASTRUCTURE ONLY (CPU oracle; never linked into,
 * called by, or shipped with the product).  Only tests/, __graft_entry__.smoke()
 * and bench.py may load it, and only as the checker.
 *
 * Plain-C restatement of the evaluation the reference runs on fused runs:
 * scripts/06_eval_fusion.py:42-49,52-140 -> IREvaluator.evaluate
 * (src/evaluation/ir_evaluator.py:51-86) -> ir_measures (>=0.3.3,
 * requirements.txt:15; not installed here) -> its default trec_eval backend.
 * Restated from trec_eval 9.x's published behaviour (parity vs the library is
 * unpinned; tests pin this file with hand-worked answers):
 *  - form_res_rels: a query's retrieved documents are sorted by score
 *    descending, ties by docno descending (comparator returns
 *    strcmp(b->docno, a->docno)); docids here are interned in docno order;
 *  - relevance_level 1: relevant = rel >= 1;
 *  - ndcg_cut.k: sum over ranks i < k of gain / log2(i + 2), gain = rel (rel >
 *    0), divided by the same sum over the judged gains sorted descending;
 *  - P_k = relevant in the top k / k; recall_k = relevant in the top k /
 *    judged relevant; recip_rank (cut k) = 1 / (i + 1) of the first relevant
 *    rank i < k; map = sum over relevant ranks i of (relevant so far) / (i + 1),
 *    divided by judged relevant;
 *  - a query without retrieved documents or without qrels is not evaluated (NaN).
 * Runs read back from a .res file carry the "%.6f" scores write_runfile
 * printed (src/fusion.py:491): text != 0 rounds every score through
 * snprintf("%.6f") first, as that round trip does.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

enum { E_NDCG = 0, E_RR, E_R, E_P, E_AP };

typedef struct {
  double s;
  uint32_t d;
} ranked_t;

static int cmp_trec(const void* a, const void* b) {
  const ranked_t* x = (const ranked_t*)a;
  const ranked_t* y = (const ranked_t*)b;
  if (x->s > y->s) return -1;
  if (x->s < y->s) return 1;
  return (y->d > x->d) - (y->d < x->d);  /* docno descending */
}

static int cmp_int_desc(const void* a, const void* b) {
  const int x = *(const int*)a, y = *(const int*)b;
  return (y > x) - (y < x);
}

static double as_text(double s) {
  char buf[64];
  snprintf(buf, sizeof buf, "%.6f", s);
  return strtod(buf, NULL);
}

int oracle_eval(int64_t n_queries, const int64_t* off, const uint32_t* docid,
                const double* score, int text, const int64_t* qrel_off,
                const uint32_t* qrel_docid, const int32_t* qrel_rel, int n_metrics,
                const int32_t* kind, const int32_t* cut, double* out) {
  for (int64_t q = 0; q < n_queries; ++q) {
    double* o = out + q * n_metrics;
    const int64_t a = off[q], n = off[q + 1] - off[q];
    const int64_t qa = qrel_off[q], nq = qrel_off[q + 1] - qrel_off[q];
    if (n <= 0 || nq <= 0) {
      for (int t = 0; t < n_metrics; ++t) o[t] = NAN;
      continue;
    }
    ranked_t* r = (ranked_t*)malloc(sizeof(ranked_t) * (size_t)n);
    int* rel = (int*)malloc(sizeof(int) * (size_t)n);
    int* gains = (int*)malloc(sizeof(int) * (size_t)nq);
    if (!r || !rel || !gains) return 1;
    for (int64_t i = 0; i < n; ++i) {
      r[i].s = text ? as_text(score[a + i]) : score[a + i];
      if (r[i].s == 0.0) r[i].s = 0.0;
      r[i].d = docid[a + i];
    }
    qsort(r, (size_t)n, sizeof(ranked_t), cmp_trec);
    int num_rel = 0, ng = 0;
    for (int64_t j = 0; j < nq; ++j) {
      if (qrel_rel[qa + j] >= 1) ++num_rel;
      if (qrel_rel[qa + j] > 0) gains[ng++] = qrel_rel[qa + j];
    }
    qsort(gains, (size_t)ng, sizeof(int), cmp_int_desc);
    for (int64_t i = 0; i < n; ++i) {
      rel[i] = 0;
      for (int64_t j = 0; j < nq; ++j)
        if (qrel_docid[qa + j] == r[i].d) { rel[i] = qrel_rel[qa + j]; break; }
    }
    for (int t = 0; t < n_metrics; ++t) {
      const int k = cut[t];
      double v = 0.0;
      if (kind[t] == E_NDCG) {
        double dcg = 0.0, idcg = 0.0;
        for (int64_t i = 0; i < n && i < k; ++i)
          if (rel[i] > 0) dcg += (double)rel[i] / log2((double)i + 2.0);
        for (int i = 0; i < ng && i < k; ++i) idcg += (double)gains[i] / log2((double)i + 2.0);
        v = idcg > 0.0 ? dcg / idcg : 0.0;
      } else if (kind[t] == E_RR) {
        for (int64_t i = 0; i < n && i < k; ++i)
          if (rel[i] >= 1) { v = 1.0 / (double)(i + 1); break; }
      } else if (kind[t] == E_R || kind[t] == E_P) {
        int hit = 0;
        for (int64_t i = 0; i < n && i < k; ++i) hit += rel[i] >= 1;
        if (kind[t] == E_R) v = num_rel > 0 ? (double)hit / (double)num_rel : 0.0;
        else v = (double)hit / (double)k;
      } else {
        double s = 0.0;
        int so_far = 0;
        for (int64_t i = 0; i < n; ++i)
          if (rel[i] >= 1) s += (double)(++so_far) / (double)(i + 1);
        v = num_rel > 0 ? s / (double)num_rel : 0.0;
      }
      o[t] = v;
    }
    free(r);
    free(rel);
    free(gains);
  }
  return 0;
}
