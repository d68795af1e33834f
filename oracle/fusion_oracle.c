/*
 * fusion_oracle.c — TEST INFRASTRUCTURE ONLY (CPU oracle; never linked into,
 * called by, or shipped with the product).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it, and only as the checker.
 *
 * Plain-C restatement of the reference fusion path, written as the reference's
 * own loops run (sequential dict accumulation), NOT as the GPU kernel works:
 *
 *  - weighted_combsum / weighted_combmnz / weighted_rrf: src/fusion.py:237-380.
 *    For each query, for each ranker in runs order, for each row in file order
 *    (W-RRF: rows sorted by the rank column, :372), doc_scores[docno] +=
 *    w * score (:273) | w / (k + rank) (:374); W-CombMNZ multiplies by the row
 *    count (:327).  Output order = dict insertion (first-seen) order.
 *  - combsum / combmnz / rrf via ranx (src/fusion.py:170-230; ranx>=0.3.16, not
 *    installed here — restated from its published semantics):
 *    per run, per query min-max normalisation (s - min) / max(max - min, 1e-9)
 *    (ranx's "avoid division by zero" denominator; a constant list gives 0); CombSUM = sum over runs in order; CombMNZ = sum * #runs;
 *    RRF = sum of 1 / (k + rank), rank = 1-based position after a stable sort
 *    of the run's list by normalised score, descending.
 *  - write_runfile / _ranx_to_dict ordering (src/fusion.py:475, :488): stable
 *    sort by fused score descending over first-seen order.
 *
 * Inputs use the same CSR layout as the product (include/qppfuse.h) so tests
 * can feed both the same buffers.  Scores are doubles.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ranx min-max denominator: max(max - min, 1e-9) (NaN stays NaN). */
static double ranx_den(double mx, double mn) {
  const double d = mx - mn;
  return d < 1e-9 ? 1e-9 : d;
}

enum { M_COMBSUM = 0, M_COMBMNZ, M_RRF, M_WCOMBSUM, M_WCOMBMNZ, M_WRRF };

typedef struct {
  uint32_t* keys;
  int32_t* vals;
  uint32_t cap;
} dict_t;

static uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

/* docid -> first-seen index; returns index (inserting when absent). */
static int32_t dict_get_or_add(dict_t* d, uint32_t key, int32_t next) {
  uint32_t h = hash32(key) & (d->cap - 1);
  for (;;) {
    if (d->vals[h] < 0) { d->keys[h] = key; d->vals[h] = next; return next; }
    if (d->keys[h] == key) return d->vals[h];
    h = (h + 1) & (d->cap - 1);
  }
}

typedef struct { double s; int32_t i; } item_t;

/* stable merge sort of items by score descending (ties: smaller i first) */
static void msort(item_t* a, item_t* tmp, int64_t n) {
  if (n < 2) return;
  int64_t h = n / 2;
  msort(a, tmp, h);
  msort(a + h, tmp, n - h);
  int64_t i = 0, j = h, k = 0;
  while (i < h && j < n) {
    /* take from the right only if strictly greater: keeps stability */
    if (a[j].s > a[i].s) tmp[k++] = a[j++];
    else tmp[k++] = a[i++];
  }
  while (i < h) tmp[k++] = a[i++];
  while (j < n) tmp[k++] = a[j++];
  memcpy(a, tmp, (size_t)n * sizeof(item_t));
}

/*
 * Fuse every query.  method: M_*.  rank: nullable (W-RRF rank column; NULL =
 * position + 1).  weights[Q*R] nullable for unweighted methods.  Outputs as the
 * product's qf_fuse: union_docid in first-seen order, union_count, and for the
 * method the sorted (perm, fused) pairs at the query's base offset.
 * Returns 0, or -1 on allocation failure.
 */
int oracle_fuse(int64_t Q, int32_t R, const int64_t* list_off, const uint32_t* docid,
                const double* score, const int32_t* rank, const double* weights, int32_t method,
                int32_t rrf_k, uint32_t* union_docid, int32_t* union_count, uint32_t* perm,
                double* fused) {
  int64_t maxn = 0;
  for (int64_t q = 0; q < Q; ++q) {
    int64_t n = list_off[(q + 1) * R] - list_off[q * R];
    if (n > maxn) maxn = n;
  }
  uint32_t cap = 16;
  while (cap < 2 * (uint64_t)maxn + 2) cap <<= 1;
  dict_t d = {malloc(cap * sizeof(uint32_t)), malloc(cap * sizeof(int32_t)), cap};
  double* acc = malloc((size_t)(maxn + 1) * sizeof(double));
  int32_t* cnt = malloc((size_t)(maxn + 1) * sizeof(int32_t));
  item_t* items = malloc((size_t)(maxn + 1) * sizeof(item_t));
  item_t* tmp = malloc((size_t)(maxn + 1) * sizeof(item_t));
  int32_t* order = malloc((size_t)(maxn + 1) * sizeof(int32_t));
  if (!d.keys || !d.vals || !acc || !cnt || !items || !tmp || !order) return -1;

  for (int64_t q = 0; q < Q; ++q) {
    const int64_t base = list_off[q * R];
    for (uint32_t i = 0; i < cap; ++i) d.vals[i] = -1;
    int32_t U = 0;
    for (int32_t r = 0; r < R; ++r) {
      const int64_t a = list_off[q * R + r], b = list_off[q * R + r + 1];
      const int64_t n = b - a;
      const double w = weights ? weights[q * R + r] : 1.0;
      /* row visiting order within the list */
      for (int64_t i = 0; i < n; ++i) order[i] = (int32_t)i;
      double mn = 0.0, mx = 0.0;
      if (method <= M_RRF && n > 0) {
        mn = mx = score[a];
        for (int64_t i = 1; i < n; ++i) {
          if (score[a + i] < mn) mn = score[a + i];
          if (score[a + i] > mx) mx = score[a + i];
        }
      }
      if (method == M_RRF) { /* ranx rank: stable sort by normalised score desc */
        for (int64_t i = 0; i < n; ++i) {
          const double den = ranx_den(mx, mn);
          items[i].s = den > 0.0 ? (score[a + i] - mn) / den : 0.0;
          items[i].i = (int32_t)i;
        }
        msort(items, tmp, n);
        for (int64_t i = 0; i < n; ++i) order[i] = items[i].i;
      } else if (method == M_WRRF && rank) { /* sort_values("rank") */
        for (int64_t i = 0; i < n; ++i) { items[i].s = -(double)rank[a + i]; items[i].i = (int32_t)i; }
        msort(items, tmp, n);
        for (int64_t i = 0; i < n; ++i) order[i] = items[i].i;
      }
      for (int64_t t = 0; t < n; ++t) {
        const int64_t i = order[t];
        const int32_t u = dict_get_or_add(&d, docid[a + i], U);
        if (u == U) { acc[U] = 0.0; cnt[U] = 0; union_docid[base + U] = docid[a + i]; ++U; }
        double c;
        switch (method) {
          case M_COMBSUM:
          case M_COMBMNZ: {
            const double den = ranx_den(mx, mn);
            c = den > 0.0 ? (score[a + i] - mn) / den : 0.0;
          } break;
          case M_RRF: c = 1.0 / (double)(rrf_k + t + 1); break;
          case M_WCOMBSUM:
          case M_WCOMBMNZ: c = w * score[a + i]; break;
          default: {
            const int32_t rk = rank ? rank[a + i] : (int32_t)(i + 1);
            c = w / (double)(rrf_k + rk);
          }
        }
        acc[u] += c;
        cnt[u] += 1;
      }
    }
    for (int32_t u = 0; u < U; ++u) {
      double v = acc[u];
      if (method == M_COMBMNZ || method == M_WCOMBMNZ) v = v * (double)cnt[u];
      items[u].s = v;
      items[u].i = u;
    }
    msort(items, tmp, U);
    for (int32_t i = 0; i < U; ++i) {
      perm[base + i] = (uint32_t)items[i].i;
      fused[base + i] = items[i].s;
    }
    union_count[q] = U;
  }
  free(d.keys); free(d.vals); free(acc); free(cnt); free(items); free(tmp); free(order);
  return 0;
}

/* Per-list min-max (src/retrievers/base.py:60-73). */
void oracle_minmax_per_query(const double* score, const int64_t* list_off, int64_t n_lists,
                             double* out) {
  for (int64_t l = 0; l < n_lists; ++l) {
    const int64_t a = list_off[l], b = list_off[l + 1];
    if (b <= a) continue;
    double mn = score[a], mx = score[a];
    for (int64_t i = a + 1; i < b; ++i) {
      if (score[i] < mn) mn = score[i];
      if (score[i] > mx) mx = score[i];
    }
    const double range = mx > mn ? mx - mn : 1.0;
    for (int64_t i = a; i < b; ++i) out[i] = (score[i] - mn) / range;
  }
}
