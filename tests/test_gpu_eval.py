"""qf_eval (HIP) vs the trec_eval restatement (oracle/eval_oracle.c) — needs an MI355X.

Per-query metric values are compared as IEEE doubles (bit-exact): both sum in
rank order with the same discounts.
"""
import numpy as np
import pytest
import torch

from oracle import _loader as coracle

pytestmark = pytest.mark.gpu

MEASURES = ["nDCG@5", "nDCG@10", "nDCG@20", "RR@5", "RR@10", "R@5", "R@10", "R@100", "P@10",
            "AP"]


def _qrels_for(lists_by_q, rng, n_max=6):
    offs, ds, rs = [0], [], []
    for docs in lists_by_q:
        n = int(rng.integers(0, n_max + 1))
        pick = list(rng.choice(docs, size=min(n, len(docs)), replace=False)) if len(docs) else []
        if rng.random() < 0.5:
            pick.append(0x7FFFFFF0 + int(rng.integers(0, 8)))  # judged, never retrieved
        pick = sorted(set(int(x) for x in pick))
        ds += pick
        rs += [int(rng.integers(0, 3)) for _ in pick]
        offs.append(len(ds))
    return (np.array(offs, np.int64), np.array(ds, np.uint32), np.array(rs, np.int32))


@pytest.mark.parametrize("text", [False, True])
def test_eval_of_fused_outputs_matches_oracle(gpu, text):
    from qppfuse import engine
    from qppfuse.evaluation import evaluate_device
    Q, R, K = 96, 5, 400
    off, docid, raw = engine.synth_runs(0, Q, R, K, seed=11, p_shared=0.7)
    _, micro = engine.minmax_per_query(raw, off, want_norm=False)
    methods = ["combsum", "combmnz", "rrf", "wcombsum", "wcombmnz", "wrrf"]
    w = torch.rand(Q * R, dtype=torch.float64, device=gpu)
    out = engine.fuse(off, docid, micro, R, methods, weights=w, max_entries=R * K)
    off_h = off.cpu().numpy()
    uc = out.union_count.cpu().numpy()
    ud = out.union_docid.cpu().numpy().view(np.uint32)
    rng = np.random.default_rng(3)
    lists = [ud[off_h[q * R]:off_h[q * R] + uc[q]] for q in range(Q)]
    qo, qd, qr = _qrels_for(lists, rng)
    t = lambda a: torch.from_numpy(a).to(gpu)
    got = evaluate_device(off, R, out.union_count, out.union_docid, out.perm, out.fused,
                          out.fused.shape[1], len(methods), Q,
                          (t(qo), t(qd.view(np.int32)), t(qr)), int(np.diff(qo).max()),
                          MEASURES, text_scores=text).cpu().numpy()
    perm = out.perm.cpu().numpy().view(np.uint16)
    fused = out.ranked_fused().cpu().numpy()
    for m in range(len(methods)):
        # the oracle gets plain ranked lists (docid, score) and sorts them itself
        roff = np.zeros(Q + 1, np.int64)
        roff[1:] = np.cumsum(uc)
        rdoc = np.concatenate([ud[off_h[q * R] + perm[m, off_h[q * R]:off_h[q * R] + uc[q]]]
                               for q in range(Q)])
        rsc = np.concatenate([fused[m, off_h[q * R]:off_h[q * R] + uc[q]] for q in range(Q)])
        want = coracle.evaluate(roff, rdoc, rsc, qo, qd, qr, MEASURES, text)
        np.testing.assert_array_equal(np.isnan(got[m]), np.isnan(want))
        ok = ~np.isnan(want)
        assert got[m][ok].tobytes() == want[ok].tobytes(), methods[m]


def test_ir_evaluator_on_dict_runs_with_ties(gpu):
    """Generic runs (dicts), heavy score ties, docno tie-break, means over evaluated queries."""
    from qppfuse.evaluation import IREvaluator
    rng = np.random.default_rng(5)
    run, qrels = {}, {}
    for q in range(40):
        n = int(rng.integers(0, 150))
        docs = [f"doc{int(x)}" for x in rng.choice(5000, size=n, replace=False)]
        scores = rng.choice([1.0, 0.5, 0.25, 0.125, 0.0], size=n).tolist()
        run[f"q{q}"] = list(zip(docs, scores))
        if q % 7 != 3:
            judged = docs[: int(rng.integers(0, 5))] + [f"doc{9000 + q}"]
            qrels[f"q{q}"] = {d: int(rng.integers(0, 3)) for d in judged}
    ev = IREvaluator(MEASURES)
    got = ev.evaluate(run, qrels, per_query=True)
    # oracle on the same packing (docnos sorted -> ids)
    names = sorted({d for v in run.values() for d, _ in v})
    idx = {d: i for i, d in enumerate(names)}
    qids = list(run.keys())
    off = np.zeros(len(qids) + 1, np.int64)
    docs, scs = [], []
    for i, q in enumerate(qids):
        docs += [idx[d] for d, _ in run[q]]
        scs += [s for _, s in run[q]]
        off[i + 1] = len(docs)
    qo, qd, qr = [0], [], []
    for q in qids:
        j = sorted(((idx.get(d, 0xFFFFFFFF), r) for d, r in qrels.get(q, {}).items()))
        qd += [a for a, _ in j]
        qr += [b for _, b in j]
        qo.append(len(qd))
    want = coracle.evaluate(off, np.array(docs, np.uint32), np.array(scs), np.array(qo),
                            np.array(qd, np.uint32), np.array(qr, np.int32), MEASURES)
    for t, m in enumerate(MEASURES):
        for i, q in enumerate(qids):
            if np.isnan(want[i, t]):
                assert q not in got[m]
            else:
                assert got[m][q] == want[i, t], (m, q)
    agg = ev.evaluate(run, qrels)
    for t, m in enumerate(MEASURES):
        col = want[:, t][~np.isnan(want[:, t])]
        assert agg[m] == pytest.approx(col.mean(), rel=1e-12)
