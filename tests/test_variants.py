"""Research fusion variants: ProbFuse.py and QPPrrf_argmax.py.

CPU tests cover the host halves (segment mapping, train_probfuse counting, argmax
selection) against faithful row-by-row ports of the reference scripts
(oracle/ref_port.py); GPU tests check the device fusions (QF_PROBFUSE,
QF_WRRF_MUL) against the same ports, scores compared bit for bit.
"""
import numpy as np
import pandas as pd
import pytest
import torch

from oracle import ref_port


def _runs(seed, n_q=12, rankers=("BM25", "Dense", "Splade"), n=60, pool=150, int_ids=False,
          shuffle_ranks=False):
    rng = np.random.default_rng(seed)
    runs = {}
    for ri, name in enumerate(rankers):
        rows = []
        for q in range(n_q):
            if (q + ri) % 7 == 6:
                continue  # a query missing from this run
            m = int(rng.integers(1, n))
            docs = rng.choice(pool, m, replace=False)
            sc = np.sort(np.round(rng.random(m), 6))[::-1]
            sc[m // 3: m // 3 + 3] = sc[m // 3]  # ties
            ranks = np.arange(1, m + 1)
            if shuffle_ranks:
                ranks = ranks + rng.integers(0, 3, m)  # file rank column != position
            for d, r, s in zip(docs, ranks, sc):
                rows.append((q if int_ids else str(q), "Q0", int(d) if int_ids else f"d{d}",
                             int(r), float(s), name))
        runs[name] = pd.DataFrame(rows, columns=["qid", "iter", "docno", "rank", "score",
                                                 "runid"])
    return runs


def test_segments_match_reference_formula():
    from qppfuse.variants import _segments, pos_to_segment
    for x, L in [(25, 100), (50, 100), (7, 30), (1, 1), (3, 1000)]:
        pos = np.arange(-3, 1200)
        want = [ref_port.probfuse_pos_to_segment(int(p), L, x) for p in pos]
        assert _segments(pos, L, x).tolist() == want
        assert [pos_to_segment(int(p), L, x) for p in pos] == want


@pytest.mark.parametrize("variant", ["judged", "all"])
def test_train_probfuse_matches_reference(variant):
    from qppfuse.variants import train_probfuse
    runs = _runs(1)
    rng = np.random.default_rng(2)
    qrels = {}
    for q in range(12):
        qrels[str(q)] = {f"d{d}": int(rng.integers(0, 3)) for d in rng.choice(150, 40, False)}
    got = train_probfuse(runs, qrels, x=10, L=60, variant=variant, eps=1e-6)
    want = ref_port.train_probfuse(runs, qrels, x=10, L=60, variant=variant, eps=1e-6)
    assert got == want


def test_adaptive_selection_matches_reference_loop():
    from qppfuse.variants import build_adaptive_run
    runs = _runs(3, int_ids=True)
    qpp = {str(q): {r: [float((q * 7 + i) % 5) for _ in range(3)] for i, r in enumerate(runs)}
           for q in range(12)}
    got = build_adaptive_run(qpp, runs, 1)
    # the reference loop (QPPrrf_argmax.py:33-51), spelled out
    parts = []
    for qid, rs in qpp.items():
        sel = max(rs.items(), key=lambda t: t[1][1])[0]
        parts.append(runs[sel][runs[sel]["qid"] == int(qid)])
    want = pd.concat(parts).sort_values(["qid", "score"], ascending=[True, False])
    want["rank"] = want.groupby("qid").cumcount() + 1
    pd.testing.assert_frame_equal(got, want)


def _assert_same_frame(got, want):
    assert list(got["qid"].astype(str)) == list(want["qid"].astype(str))
    assert list(got["docno"]) == list(want["docno"])
    assert got["rank"].tolist() == want["rank"].tolist()
    assert got["score"].to_numpy(np.float64).tobytes() == \
        want["score"].to_numpy(np.float64).tobytes()
    assert got["runid"].tolist() == want["runid"].tolist()


@pytest.mark.gpu
@pytest.mark.parametrize("shuffle_ranks", [False, True])
def test_probfuse_run_bit_exact(gpu, shuffle_ranks):
    from qppfuse.variants import build_probfuse_run, train_probfuse
    runs = _runs(4, shuffle_ranks=shuffle_ranks)
    rng = np.random.default_rng(5)
    qrels = {str(q): {f"d{d}": int(rng.integers(0, 2)) for d in rng.choice(150, 50, False)}
             for q in range(12)}
    P = train_probfuse(runs, qrels, x=25, L=100)
    P.pop("Splade")  # a run without probabilities contributes 0.0
    got = build_probfuse_run(runs, P, x=25, L=100, run_tag="probFuse-judged")
    want = ref_port.build_probfuse_run(runs, P, x=25, L=100, run_tag="probFuse-judged")
    _assert_same_frame(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("weighted", [False, True])
def test_rrf_mul_run_bit_exact(gpu, weighted):
    from qppfuse.variants import build_rrf_run
    runs = _runs(6, int_ids=True, shuffle_ranks=True)
    qpp = None
    if weighted:
        rng = np.random.default_rng(7)
        qpp = {str(q): {r: rng.random(13).tolist() for r in runs if (q + len(r)) % 5}
               for q in range(12)}
    got = build_rrf_run(runs, 60, qpp, 3 if weighted else None)
    want = ref_port.build_rrf_run(runs, 60, qpp, 3 if weighted else None)
    _assert_same_frame(got, want)
