"""The trec_eval restatement (oracle/eval_oracle.c) on hand-worked cases (CPU).

ir_measures / pytrec_eval are not installed, so these known answers — derived
by hand from trec_eval's definitions — pin the oracle the GPU eval is checked
against (parity with the library itself is unpinned).
"""
import math

import numpy as np
import pytest

from oracle import _loader as coracle

M = ["nDCG@10", "nDCG@1", "RR@10", "RR@1", "P@10", "R@5", "R@1", "AP"]


def _one(docs, scores, qrels, measures=M, text=False):
    off = np.array([0, len(docs)], np.int64)
    qd = np.array(sorted(qrels), np.uint32)
    qr = np.array([qrels[d] for d in sorted(qrels)], np.int32)
    return coracle.evaluate(off, np.array(docs, np.uint32), np.array(scores, np.float64),
                            np.array([0, len(qd)], np.int64), qd, qr, measures, text)[0]


def test_ties_break_by_docno_descending():
    # a=0 b=1 c=2 d=3, e=4 judged but not retrieved; b and c tie at 0.8 -> c first
    v = _one([0, 1, 2, 3], [0.9, 0.8, 0.8, 0.5], {1: 1, 2: 2, 4: 1})
    dcg = 2 / math.log2(3) + 1 / math.log2(4)
    idcg = 2 + 1 / math.log2(3) + 1 / math.log2(4)
    assert v[0] == pytest.approx(dcg / idcg, abs=0, rel=1e-15)
    assert v[1] == 0.0                      # nDCG@1: rank 0 (a) is not relevant
    assert v[2] == 0.5 and v[3] == 0.0      # RR@10, RR@1
    assert v[4] == pytest.approx(0.2)       # P@10 divides by 10
    assert v[5] == pytest.approx(2 / 3)     # R@5: 2 of 3 judged relevant
    assert v[6] == 0.0
    assert v[7] == pytest.approx((1 / 2 + 2 / 3) / 3)


def test_text_scores_tie_where_doubles_do_not():
    # 0.1234564 and 0.1234561 both print 0.123456: ties, then docno descending
    docs, sc, qrels = [5, 9], [0.1234564, 0.1234561], {5: 1}
    exact = _one(docs, sc, qrels, ["RR@10"])
    text = _one(docs, sc, qrels, ["RR@10"], text=True)
    assert exact[0] == 1.0 and text[0] == 0.5


def test_grade_levels_and_zero_rel():
    # rel 0 is judged non-relevant; gains are the rel levels
    v = _one([3, 2, 1], [3.0, 2.0, 1.0], {3: 0, 2: 3, 1: 1}, ["nDCG@3", "P@3", "AP"])
    dcg = 3 / math.log2(3) + 1 / math.log2(4)
    idcg = 3 + 1 / math.log2(3)
    assert v[0] == pytest.approx(dcg / idcg)
    assert v[1] == pytest.approx(2 / 3)
    assert v[2] == pytest.approx((1 / 2 + 2 / 3) / 2)


def test_unevaluated_queries_are_nan():
    off = np.array([0, 2, 2, 3], np.int64)           # q1 has no documents
    doc = np.array([1, 2, 7], np.uint32)
    sc = np.array([1.0, 0.5, 0.3])
    qo = np.array([0, 1, 2, 2], np.int64)            # q2 has no qrels
    qd = np.array([2, 7], np.uint32)
    qr = np.array([1, 1], np.int32)
    v = coracle.evaluate(off, doc, sc, qo, qd, qr, ["nDCG@10", "AP"])
    assert v[0, 0] == pytest.approx(1 / math.log2(3))
    assert np.isnan(v[1]).all() and np.isnan(v[2]).all()


def test_measure_parsing():
    from qppfuse.evaluation import parse_measure
    assert parse_measure("nDCG@10") == (0, 10)
    assert parse_measure("RR@5") == (1, 5)
    assert parse_measure("R@100") == (2, 100)
    assert parse_measure("P@10") == (3, 10)
    assert parse_measure("AP")[0] == 4
    with pytest.raises(ValueError):
        parse_measure("Judged@10")
    with pytest.raises(ValueError):
        parse_measure("P")


def test_pack_qrels_maps_onto_sorted_docnos():
    from qppfuse.evaluation import pack_qrels
    docnos = np.array(["d1", "d2", "d3"], dtype=object)
    qs = pack_qrels({"q1": {"d3": 1, "zz": 2, "d1": 0}, "q3": {"d2": 1}}, ["q1", "q2", "q3"],
                    docnos)
    assert qs.off.tolist() == [0, 3, 3, 4]
    assert qs.docid[:3].tolist() == [0, 2, 0xFFFFFFFF]
    assert qs.rel[:3].tolist() == [0, 1, 2]
    assert qs.max_per_query == 3
