"""The oracle pinned against the reference's own outputs (CPU).

Golden vectors come from running the reference's code (tests/golden/
make_golden.py).  Both oracle restatements — the faithful Python port and the
C oracle — must reproduce them bit for bit before they are trusted to check the
HIP kernels.
"""
import json
import math

import numpy as np
import pytest

from oracle import _loader as coracle
from oracle import ref_port, text_oracle
from tests.helpers import (csr_from_rows, decode_fused, first_seen_lists, frames_from_rows,
                           unhex)

WEIGHTED = ["wcombsum", "wcombmnz", "wrrf"]


def _case_ids(golden):
    return [c["name"] for c in golden["cases"]]


@pytest.mark.parametrize("method", WEIGHTED)
def test_python_port_matches_reference_weighted(golden, method):
    for case in golden["cases"]:
        frames = frames_from_rows(case["runs"], case["rankers"])
        got = ref_port.weighted_fusion(frames, case["qpp"], case["qpp_index"], method,
                                       case["rrf_k"])
        want = decode_fused(case["outputs"][method])
        assert list(got.keys()) == list(want.keys()), case["name"]
        for q in want:
            assert [(d, s) for d, s in got[q]] == want[q], (case["name"], q)
        assert ref_port.runfile_text(got, f"{method}-tag") == case["runfiles"][method]


@pytest.mark.parametrize("method", WEIGHTED)
def test_c_oracle_matches_reference_weighted(golden, method):
    for case in golden["cases"]:
        R = len(case["rankers"])
        qids, off, docid, score, rank, docnos = csr_from_rows(
            case["runs"], case["rankers"], by_rank=(method == "wrrf"))
        w = np.array([ref_port.qpp_weight(q, r, case["qpp"], case["qpp_index"],
                                          case["qpp_index"] == -1)
                      for q in qids for r in case["rankers"]])
        ud, uc, perm, fused = coracle.fuse(off, docid, score, R, method, case["rrf_k"],
                                           weights=w, rank=rank)
        got = first_seen_lists(qids, docnos, ud, uc, perm, fused, off, R)
        want = decode_fused(case["outputs"][method])
        for q in want:
            assert got[q] == want[q], (case["name"], method, q)


@pytest.mark.parametrize("pair", [("combsum", "wcombsum"), ("combmnz", "wcombmnz"),
                                  ("rrf", "wrrf")])
def test_unweighted_equals_unit_weighted_on_norm_runs(golden, pair):
    """ranx CombSUM/CombMNZ/RRF == W-* with all weights 1 on .norm.res lists.

    ranx is not installed; this pins the unweighted restatement (min-max is the
    identity on per-query min-max normalised lists, sums run in runs order) to
    the reference's own weighted loops.
    """
    un, wt = pair
    for case in golden["cases"]:
        if case["name"] != "unit_weights":
            continue
        frames = frames_from_rows(case["runs"], case["rankers"])
        got = ref_port.ranx_fusion(frames, un, case["rrf_k"])
        want = decode_fused(case["outputs"][wt])
        for q in want:
            ranked = sorted(want[q], key=lambda x: x[1], reverse=True)
            assert got[q] == ranked, (un, q)
        R = len(case["rankers"])
        qids, off, docid, score, rank, docnos = csr_from_rows(case["runs"], case["rankers"])
        ud, uc, perm, fused = coracle.fuse(off, docid, score, R, un, case["rrf_k"])
        for qi, q in enumerate(qids):
            b, n = off[qi * R], uc[qi]
            got_c = list(zip(docnos[ud[b + perm[b:b + n].astype(int)]].tolist(),
                             fused[b:b + n].tolist()))
            assert got_c == sorted(want[q], key=lambda x: x[1], reverse=True), (un, q)


def test_normalize_qpp_port(golden):
    g = golden["normalize_qpp"]
    raw = {q: [unhex(v) for v in r] for q, r in g["raw"].items()}
    got = ref_port.normalize_qpp(raw, "minmax")
    for q, row in g["norm"].items():
        assert [float(v) for v in got[q]] == [unhex(v) for v in row]


def test_normalize_scores_port_and_c_oracle(golden):
    for case in golden["normalize_scores"]:
        src = [(d, unhex(s), r) for d, s, r in case["in"]]
        want = [(d, unhex(s), r) for d, s, r in case["out"]]
        assert ref_port.normalize_scores(src) == want
        if src:
            out = coracle.minmax_per_query(np.array([s for _, s, _ in src]),
                                           np.array([0, len(src)]))
            assert out.tolist() == [s for _, s, _ in want]


def test_error_semantics_port(golden):
    for e in golden["errors"]:
        frames = frames_from_rows(e["runs"], ["BGE", "BM25", "Splade"])
        with pytest.raises(Exception) as exc:
            ref_port.weighted_fusion(frames, e["qpp"], e["qpp_index"], "wcombsum")
        assert [type(exc.value).__name__, str(exc.value)] == e["error"]


@pytest.mark.parametrize("ds", ["scifact", "nq"])
def test_text_columns_match_committed_qpp(ds):
    """Columns 7-8 of the committed .qpp files (text-only predictors) reproduce exactly."""
    from tests.conftest import GOLDEN
    fx = json.loads((GOLDEN / f"qpp_textcols_{ds}.json").read_text())
    feats = [text_oracle.text_features(t) for t in fx["text"]]
    for col, j in (("col7", 1), ("col8", 2)):
        vals = np.array([f[j] for f in feats])
        lo, hi = vals.min(), vals.max()
        norm = (vals - lo) / (hi - lo if hi > lo else 1.0)
        got = [f"{v:.6f}" for v in norm]
        assert got == fx[col], col
    assert fx["col11"] == fx["col12"]


def test_qpp_known_answers():
    # NQC of [0.9, 0.7, 0.5] (float32 inputs): population variance.
    xs = [float(np.float32(v)) for v in (0.9, 0.7, 0.5)]
    mean = sum(xs) / 3
    nqc = sum((x - mean) ** 2 for x in xs) / 3
    got = ref_port.java_qpp(1, 0.0, 0.0, [0.9, 0.7, 0.5])
    assert math.isclose(got["nqc"], nqc, rel_tol=1e-15)
    assert math.isclose(got["nqc"], 0.02666666, rel_tol=1e-5)
    assert got["dense-qpp"] == got["dense-qpp-m"] == pytest.approx(math.log(1 + 1 / (xs[0] - xs[2])))
    assert ref_port.java_qpp(3, 1.0, 2.0, []) == {}
    one = ref_port.java_qpp(2, 1.0, 2.0, [0.5])
    assert one["SigmaMax"] == one["SigmaX"] == one["RSD"] == one["cumnqc"] == 0.0


def test_c_and_python_qpp_restatements_agree():
    rng = np.random.default_rng(7)
    lists = [rng.normal(5, 3, n) for n in (1, 2, 3, 7, 50, 64, 100)]
    lists += [np.sort(rng.uniform(-12, -0.5, 40))[::-1], np.full(10, 0.25),
              np.sort(rng.gamma(2, 6, 80))[::-1]]
    lists = [np.sort(l)[::-1] for l in lists]
    off = np.cumsum([0] + [len(l) for l in lists])
    flat = np.concatenate(lists)
    nt = np.arange(len(lists), dtype=np.int32) % 5
    mi = np.linspace(0.5, 2.0, len(lists))
    ai = np.linspace(1.0, 3.0, len(lists))
    c = coracle.qpp_raw(flat, off, nt, mi, ai)
    for i, l in enumerate(lists):
        py = ref_port.java_qpp(int(nt[i]), float(mi[i]), float(ai[i]), l.tolist())
        row = [py[n] for n in ref_port.QPP_NAMES]
        np.testing.assert_allclose(c[i], row, rtol=1e-13, atol=1e-15)
