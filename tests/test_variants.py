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


# ---------------------------------------------- 10_oracle_baseline.py -------

@pytest.mark.parametrize("s,want", [
    ("ndcg@10", "nDCG@10"), ("nDCG@5", "nDCG@5"), ("ndcg", "nDCG@10"), ("map", "AP"),
    ("AP", "AP"), ("mrr@10", "RR@10"), ("rr", "RR@10"), ("RR@3", "RR@3"), ("recall@100", "R@100"),
    ("recall", "R@10"), ("r@5", "R@5"), (" NDCG@20 ", "nDCG@20")])
def test_parse_metric(s, want):
    from qppfuse.variants import parse_metric
    assert parse_metric(s) == want


def test_parse_metric_unknown():
    from qppfuse.variants import parse_metric
    with pytest.raises(ValueError, match="Unknown metric"):
        parse_metric("p@10")


def test_oracle_selection_rules():
    """compute_oracle_run's loop (10_oracle_baseline.py:171-199): judged qids only, in
    sorted order; strictly greater wins (first ranker in dict order on ties); a 0.0
    score still beats the initial -1; a query missing from every ranker is dropped."""
    from qppfuse.variants import _select_best
    runs = {"A": {"1": [("a", 1.0)], "2": [("b", 1.0)], "3": [("c", 1.0)], "9": [("z", 1.0)]},
            "B": {"1": [("d", 1.0)], "2": [("e", 1.0)], "4": [("f", 1.0)]}}
    qrels = {"1": {"a": 1}, "2": {"b": 1}, "3": {"x": 1}, "4": {"f": 1}, "5": {"y": 1}}
    scores = {"A": {"1": 0.5, "2": 0.25, "3": 0.0}, "B": {"1": 0.5, "2": 0.75, "4": 1.0}}
    oracle_run, sel = _select_best(runs, qrels, scores)
    assert sel == {"1": "A", "2": "B", "3": "A", "4": "B"}
    assert list(oracle_run) == ["1", "2", "3", "4"]
    assert oracle_run["2"] == [("e", 1.0)]


def test_analyze_oracle_selections():
    from qppfuse.variants import analyze_oracle_selections
    sel = {"1": "A", "2": "B", "3": "A"}
    pq = {"A": {"1": 0.6, "3": 0.5}, "B": {"1": 0.3, "2": 0.4}, "C": {"1": 0.3, "2": 0.2}}
    a = analyze_oracle_selections(sel, pq)
    assert a["selection_counts"] == {"A": 2, "B": 1}
    assert a["selection_percentages"] == {"A": 2 / 3 * 100, "B": 1 / 3 * 100}
    assert a["n_queries"] == 3
    # q1: (0.6 - 0.3) / 0.3; q2: (0.4 - 0.1) / 0.1; q3: others average 0 -> skipped
    gains = [(0.6 - 0.3) / 0.3 * 100, (0.4 - np.mean([0.0, 0.2])) / np.mean([0.0, 0.2]) * 100]
    assert a["avg_improvement_over_others"] == pytest.approx(np.mean(gains))
    assert a["max_improvement"] == pytest.approx(max(gains))


def test_load_all_runs(tmp_path):
    from qppfuse.variants import load_all_runs
    (tmp_path / "BM25.res").write_text("1 Q0 a 2 0.5 t\n1 Q0 b 1 0.9 t\n2 Q0 c 1 0.1 t\n")
    (tmp_path / "BM25.norm.res").write_text("1 Q0 a 1 1.0 t\n")
    (tmp_path / "Dense.res").write_text("1 Q0 b 1 0.3 t\n1 Q0 a 2 0.3 t\n")
    raw = load_all_runs(tmp_path)
    assert list(raw) == ["BM25", "Dense"]
    assert raw["BM25"] == {"1": [("b", 0.9), ("a", 0.5)], "2": [("c", 0.1)]}
    assert raw["Dense"]["1"] == [("b", 0.3), ("a", 0.3)]  # stable on equal scores
    assert load_all_runs(tmp_path, use_normalized=True) == {"BM25": {"1": [("a", 1.0)]}}


def _oracle_metric(run, qrels, measure):
    """Per-query values of one {qid: [(docno, score)]} run from the trec_eval restatement."""
    from oracle import _loader as coracle
    names = sorted({d for v in run.values() for d, _ in v} |
                   {d for v in qrels.values() for d in v})
    idx = {d: i for i, d in enumerate(names)}
    qids = list(run)
    off, docs, scs = [0], [], []
    for q in qids:
        dd = {}
        for d, s in run[q]:
            dd[d] = s
        docs += [idx[d] for d in dd]
        scs += list(dd.values())
        off.append(len(docs))
    qo, qd, qr = [0], [], []
    for q in qids:
        j = sorted((idx[d], r) for d, r in qrels.get(q, {}).items())
        qd += [a for a, _ in j]
        qr += [b for _, b in j]
        qo.append(len(qd))
    v = coracle.evaluate(np.array(off, np.int64), np.array(docs, np.uint32), np.array(scs),
                         np.array(qo, np.int64), np.array(qd, np.uint32), np.array(qr, np.int32),
                         [measure])[:, 0]
    return {q: float(x) for q, x in zip(qids, v) if not np.isnan(x)}


def _oracle_runs(seed, n_q=30, rankers=("BM25", "BGE", "Splade")):
    rng = np.random.default_rng(seed)
    runs, qrels = {}, {}
    for q in range(n_q):
        if q % 9 != 4:
            qrels[str(q)] = {f"d{int(d)}": int(rng.integers(0, 3))
                             for d in rng.choice(300, int(rng.integers(1, 8)), replace=False)}
    for ri, r in enumerate(rankers):
        runs[r] = {}
        for q in range(n_q + 3):
            if (q + ri) % 8 == 7:
                continue
            m = int(rng.integers(1, 120))
            docs = [f"d{int(d)}" for d in rng.choice(300, m, replace=False)]
            sc = rng.choice([1.0, 0.75, 0.5, 0.25], m) if q % 3 == 0 else rng.random(m)
            runs[r][str(q)] = sorted(zip(docs, sc.tolist()), key=lambda t: -t[1])
    return runs, qrels


@pytest.mark.gpu
@pytest.mark.parametrize("metric", ["ndcg@10", "map", "mrr@10", "recall@100"])
def test_oracle_baseline_on_device(gpu, metric):
    from qppfuse.variants import (_select_best, compute_oracle_run, compute_per_query_scores,
                                  evaluate_run, parse_metric)
    runs, qrels = _oracle_runs(8)
    name = parse_metric(metric)
    got = compute_per_query_scores(runs, qrels, name)
    want = {r: _oracle_metric(run, qrels, name) for r, run in runs.items()}
    assert got == want
    oracle_run, sel = compute_oracle_run(runs, qrels, name)
    assert (oracle_run, sel) == _select_best(runs, qrels, want)
    ms = ["nDCG@5", "nDCG@10", "RR@10", "R@100", "AP"]
    ev = evaluate_run(oracle_run, qrels, ms)
    for m in ms:
        col = list(_oracle_metric(oracle_run, qrels, m).values())
        assert ev[m] == pytest.approx(np.mean(col), rel=1e-12)


def test_parse_measures_like_the_scripts():
    """ProbFuse.py:198-222 and QPPrrf_argmax.py:119-131's measure lists."""
    from qppfuse.variants import Measure, parse_argmax_measures, parse_measures
    assert parse_measures(["map", "ndcg@10", "recip_rank", "p5", "ndcg", "rr"]) == [
        Measure("AP(rel=2)", "AP", 2), Measure("nDCG@10", "nDCG@10"), Measure("RR", "RR"),
        Measure("P@5", "P@5"), Measure("nDCG", "nDCG"), Measure("RR", "RR")]
    for bad in ("mrr", "pX", "recall@10"):
        with pytest.raises(ValueError, match="Unsupported metric"):
            parse_measures([bad])
    # the argmax script skips what it does not know, and only takes "ndcg@10" names
    assert parse_argmax_measures(["map", "NDCG@10", "recip_rank", "p10", "ndcg@5"]) == [
        Measure("AP(rel=2)", "AP", 2), Measure("nDCG@10", "nDCG@10"), Measure("RR", "RR")]


@pytest.mark.gpu
def test_experiment_table_with_rel2_ap(gpu):
    """experiment(): one row per run, the mean of every measure; AP(rel=2) is AP
    with grades below 2 non-relevant (judged), checked against the trec_eval
    restatement on the leveled qrels."""
    from qppfuse.variants import experiment, parse_measures
    runs, qrels = _oracle_runs(5)
    ms = parse_measures(["map", "ndcg@10", "recip_rank", "p10"])
    table = experiment(list(runs.values()), qrels, ms, list(runs))
    assert list(table.columns) == ["name", "AP(rel=2)", "nDCG@10", "RR", "P@10"]
    assert table["name"].tolist() == list(runs)
    lev = {q: {d: (g if g >= 2 else 0) for d, g in docs.items()} for q, docs in qrels.items()}
    for i, (name, run) in enumerate(runs.items()):
        ap2 = list(_oracle_metric(run, lev, "AP").values())
        assert table.loc[i, "AP(rel=2)"] == pytest.approx(np.mean(ap2), rel=1e-12)
        for col, m in (("nDCG@10", "nDCG@10"), ("RR", "RR"), ("P@10", "P@10")):
            want = list(_oracle_metric(run, qrels, m).values())
            assert table.loc[i, col] == pytest.approx(np.mean(want), rel=1e-12)
    # AP(rel=2) differs from AP at rel 1 on these qrels (grades 1 and 2 both occur)
    ap1 = experiment(list(runs.values()), qrels, ["AP"], list(runs))["AP"].to_numpy()
    assert not np.allclose(ap1, table["AP(rel=2)"].to_numpy())
