// qf_eval.hip — IR evaluation of ranked runs on gfx950 (trec_eval semantics).
//
// Replaces the evaluation step of scripts/06_eval_fusion.py:52-140, which reads
// every fused .res file back (scores as the "%.6f" text write_runfile printed,
// src/fusion.py:491) and hands it to ir_measures (src/evaluation/
// ir_evaluator.py:51-86), whose trec_eval backend ranks a query's documents by
// score descending, ties by docno descending (strcmp), and computes
//   nDCG@k  Σ_{rank<k} gain / log2(rank + 2)  ÷  the same over the qrels' gains
//           sorted descending (gain = rel level, rel > 0)
//   RR@k    1 / (rank + 1) of the first relevant document within the cut
//   R@k     relevant retrieved within the cut / relevant judged
//   P@k     relevant retrieved within the cut / k
//   AP      Σ over relevant retrieved, in rank order, of precision at its rank
//           / relevant judged
// (relevant = rel >= 1; ranks 0-based).  Docids are interned in docno string
// order, so "docno descending" is "docid descending".
//
// eval_kernel — one wavefront per (run, query).  The run's list is already
// sorted by score descending (the fusion kernel's output), so the trec_eval
// order differs from it only inside groups of equal scores — equal "%.6f"
// values for runs read back from text — which are contiguous.  The wave finds the relevant documents (binary search of every
// listed docid in the query's sorted qrels), and for each one its trec_eval
// rank = start of its equal-value group + documents of the group with a larger
// docid.  All metrics follow from the ranks of the relevant documents; the
// sums run in rank order on one lane, as trec_eval's loops do.
#include "../../include/qppfuse.h"
#include "qf_common.h"
#include "qf_internal.h"
#include "qf_log2_table.h"

namespace qf {

constexpr int kEvalWaves = 4;

struct EvalRun {
  const double* score;
  const uint16_t* perm;
  const uint32_t* docid;
  int text;
  __device__ __forceinline__ uint32_t doc(int64_t base, int i) const {
    return perm ? docid[base + perm[base + i]] : docid[base + i];
  }
  // equality class of a score: the "%.6f" value write_runfile prints (text
  // runs), else the double itself (-0.0 == +0.0)
  __device__ __forceinline__ long long micro(int64_t base, int i) const {
    // qf_fuse output (perm given): its scores are by u, ranked through perm
    const double s = perm ? score[base + perm[base + i]] : score[base + i];
    return text ? round6(s) : (long long)f64_asc_key(s);
  }
};

__device__ __forceinline__ double discount(int rank) {
  return rank < kLog2RankN ? kLog2Rank[rank] : log2((double)rank + 2.0);
}

__global__ __launch_bounds__(64 * kEvalWaves) void eval_kernel(EvalParams p) {
  __shared__ int s_rank[kEvalWaves][kEvalMaxRel];
  __shared__ int s_rel[kEvalWaves][kEvalMaxRel];
  __shared__ int s_ideal[kEvalWaves][kEvalMaxRel];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t gw = block_id() * kEvalWaves + w;
  if (gw >= p.n_queries * (int64_t)p.n_runs) return;
  const int m = (int)(gw / p.n_queries);
  const int64_t q = gw % p.n_queries;
  double* out = p.out + gw * p.n_metrics;
  const int64_t base = p.q_base[q * p.base_stride];
  const int64_t n64 = p.q_count ? (int64_t)p.q_count[q] : p.q_base[(q + 1) * p.base_stride] - base;
  const int64_t qa = p.qrel_off[q], qb = p.qrel_off[q + 1];
  if (n64 <= 0 || qb <= qa) {  // not in the run or not in the qrels: not evaluated
    if (lane < p.n_metrics) out[lane] = __builtin_nan("");
    return;
  }
  const int n = (int)n64;
  const EvalRun run{p.score + (int64_t)m * p.out_stride,
                    p.perm ? p.perm + (int64_t)m * p.out_stride : nullptr,
                    p.docid + (p.perm ? 0 : (int64_t)m * p.out_stride), p.text_scores};
  // ---- judged relevant documents --------------------------------------------
  int num_rel = 0;
  for (int64_t c = qa; c < qb; c += 64) {
    const bool r = c + lane < qb && p.qrel_rel[c + lane] >= 1;
    num_rel += __popcll(ballot(r));
  }
  // ---- retrieved relevant documents, in list order ----------------------------
  int nf = 0;
  for (int c = 0; c < n; c += 64) {
    const int i = c + lane;
    int rel = 0;
    if (i < n) {
      const uint32_t d = run.doc(base, i);
      int64_t lo = qa, hi = qb;  // qrel_docid sorted ascending within the query
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (p.qrel_docid[mid] < d) lo = mid + 1;
        else hi = mid;
      }
      if (lo < qb && p.qrel_docid[lo] == d) rel = p.qrel_rel[lo];
    }
    const uint64_t b = ballot(rel > 0);
    const int pos = nf + (int)mbcnt(b);
    if (rel > 0 && pos < kEvalMaxRel) {
      s_rank[w][pos] = i;  // list position for now
      s_rel[w][pos] = rel;
    }
    nf += __popcll(b);
  }
  nf = min(nf, kEvalMaxRel);  // qf_eval rejects qrels larger than kEvalMaxRel
  // ---- trec_eval rank of each: its "%.6f" group start + larger docids inside ---
  for (int f = 0; f < nf; ++f) {
    const int pidx = s_rank[w][f];
    const long long mv = run.micro(base, pidx);
    const uint32_t dp = run.doc(base, pidx);
    int g = pidx;  // group start
    while (g > 0) {
      const int j = g - 1 - lane;
      const bool ne = j >= 0 && run.micro(base, j) != mv;
      const uint64_t b = ballot(ne || j < 0);
      if (b) { g -= __ffsll((unsigned long long)b) - 1; break; }
      g -= 64;
    }
    if (g < 0) g = 0;
    int e = pidx + 1;  // group end
    while (e < n) {
      const int j = e + lane;
      const bool ne = j >= n || run.micro(base, j) != mv;
      const uint64_t b = ballot(ne);
      if (b) { e += __ffsll((unsigned long long)b) - 1; break; }
      e += 64;
    }
    int larger = 0;
    for (int c = g; c < e; c += 64) {
      const int j = c + lane;
      larger += __popcll(ballot(j < e && run.doc(base, j) > dp));
    }
    if (lane == 0) s_rank[w][f] = g + larger;
  }
  if (lane != 0) return;
  // ---- lane 0: relevant documents in rank order, judged gains largest first,
  // then the metrics ------------------------------------------------------------
  int* rk = s_rank[w];
  int* rl = s_rel[w];
  for (int a = 1; a < nf; ++a) {  // insertion sort by rank (ranks are distinct)
    const int r0 = rk[a], v0 = rl[a];
    int b = a - 1;
    while (b >= 0 && rk[b] > r0) { rk[b + 1] = rk[b]; rl[b + 1] = rl[b]; --b; }
    rk[b + 1] = r0;
    rl[b + 1] = v0;
  }
  int* ideal = s_ideal[w];
  int ni = 0;
  for (int64_t c = qa; c < qb && ni < kEvalMaxRel; ++c) {
    const int r = p.qrel_rel[c];
    if (r <= 0) continue;
    int b = ni - 1;
    while (b >= 0 && ideal[b] < r) { ideal[b + 1] = ideal[b]; --b; }
    ideal[b + 1] = r;
    ++ni;
  }
  for (int t = 0; t < p.n_metrics; ++t) {
    const int kind = p.kind[t], k = p.cut[t];
    double v = 0.0;
    if (kind == QF_EVAL_NDCG) {
      double dcg = 0.0;
      for (int f = 0; f < nf && rk[f] < k; ++f) dcg += (double)rl[f] / discount(rk[f]);
      double idcg = 0.0;
      for (int i = 0; i < ni && i < k; ++i) idcg += (double)ideal[i] / discount(i);
      v = idcg > 0.0 ? dcg / idcg : 0.0;
    } else if (kind == QF_EVAL_RR) {
      if (nf > 0 && rk[0] < k) v = 1.0 / (double)(rk[0] + 1);
    } else if (kind == QF_EVAL_R || kind == QF_EVAL_P) {
      int hit = 0;
      while (hit < nf && rk[hit] < k) ++hit;
      if (kind == QF_EVAL_R) v = num_rel > 0 ? (double)hit / (double)num_rel : 0.0;
      else v = (double)hit / (double)k;
    } else {  // QF_EVAL_AP
      double s = 0.0;
      for (int f = 0; f < nf; ++f) s += (double)(f + 1) / (double)(rk[f] + 1);
      v = num_rel > 0 ? s / (double)num_rel : 0.0;
    }
    out[t] = v;
  }
}

hipError_t eval_launch(const EvalParams& p, hipStream_t st) {
  const int64_t waves = p.n_queries * (int64_t)p.n_runs;
  if (waves == 0) return hipSuccess;
  hipLaunchKernelGGL(eval_kernel, grid_for((waves + kEvalWaves - 1) / kEvalWaves),
                     dim3(64 * kEvalWaves), 0, st, p);
  return hipGetLastError();
}

}  // namespace qf
