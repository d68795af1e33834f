"""The evaluator's run flattening (qppfuse.evaluation._run_arrays_flat) — CPU.

scripts/06_eval_fusion.py:42-49 hands IREvaluator.evaluate the rows of
load_run_file re-sorted per query; those rows hold the very str objects of the
docno table the native loader decoded, which the flattening codes by identity.  The
arrays must equal the string path's (pandas.factorize over str) in every case: ties,
lists not in score order, a run whose rows hold other str objects (the identity
path declines), and a repeated docno (both decline: the dict semantics decide).
"""
import numpy as np
import pytest

from qppfuse import evaluation as E
from qppfuse import fastio
from qppfuse.data_utils import load_run_file


def _write_run(path, rng, n_q=40, k=300, repeat=False):
    lines = []
    for q in range(n_q):
        docs = rng.choice(5000, size=k, replace=False) + 5000 * q  # (q % 29 repeats a qid)
        if repeat and q == 7:
            docs[5] = docs[2]
        sc = np.round(np.sort(rng.random(k))[::-1], 3)  # %.3f: many equal scores
        for i in range(k):
            lines.append(f"q{q % 29} Q0 d{docs[i]} {i + 1} {sc[i]:.6f} tag\n")
    path.write_text("".join(lines))


def _wrapper(run):  # scripts/06_eval_fusion.py:46-49
    return {qid: sorted([(d, s) for d, s, r in docs], key=lambda x: -x[1])
            for qid, docs in run.items()}


def _both(run):
    qids = [str(k) for k in run]
    fastio.docno_tables.clear()
    want = E._run_arrays_flat(run, qids)
    return qids, want


def _assert_same(a, b):
    assert (a is None) == (b is None)
    if a is None:
        return
    assert a[0] == b[0]
    assert list(a[1]) == list(b[1])
    for x, y in zip(a[2:], b[2:]):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("order", ["wrapper", "file", "shuffled"])
def test_identity_coding_equals_string_coding(tmp_path, order):
    rng = np.random.default_rng(3)
    p = tmp_path / "r.res"
    _write_run(p, rng)
    run = load_run_file(p)
    if order == "wrapper":
        run = _wrapper(run)
    elif order == "file":
        run = {q: [(d, s) for d, s, r in rows] for q, rows in run.items()}
    else:  # lists not in score order: the lexsort decides
        run = {q: [(d, s) for d, s, r in rows][::-1] for q, rows in run.items()}
    qids = [str(k) for k in run]
    assert fastio.docno_tables, "read_run_rows registers its docno table"
    got = E._run_arrays_flat(run, qids)
    assert got is not None
    _, want = _both(run)
    _assert_same(got, want)


def test_other_str_objects_take_the_string_path(tmp_path):
    rng = np.random.default_rng(4)
    p = tmp_path / "r.res"
    _write_run(p, rng)
    run = _wrapper(load_run_file(p))
    copied = {q: [("".join(list(d)), s) for d, s in rows] for q, rows in run.items()}
    qids = [str(k) for k in copied]
    assert E._coded_by_table([it for x in copied.values() for it in x],
                             sum(map(len, copied.values()))) is None
    got = E._run_arrays_flat(copied, qids)
    _, want = _both(run)
    _assert_same(got, want)


def test_repeated_docno_declines_both_ways(tmp_path):
    rng = np.random.default_rng(5)
    p = tmp_path / "r.res"
    _write_run(p, rng, repeat=True)
    run = _wrapper(load_run_file(p))
    qids = [str(k) for k in run]
    assert E._run_arrays_flat(run, qids) is None
    _, want = _both(run)
    assert want is None


def test_non_ascii_docnos_sort_as_python_strings(tmp_path):
    """The table's Arrow sort (UTF-8 bytes) orders docnos as Python's str order (code
    points): accents, CJK, astral-plane and mixed-case ids."""
    rng = np.random.default_rng(6)
    alphabet = ["a", "B", "é", "É", "z", "中", "文", "\U0001F600", "ß", "0", "_"]
    lines = []
    for q in range(12):
        docs = {"".join(rng.choice(alphabet, size=int(rng.integers(1, 6)))) + f"{q}_{i}"
                for i in range(80)}
        for i, d in enumerate(sorted(docs)):
            lines.append(f"q{q} Q0 {d} {i + 1} {rng.random():.6f} t\n")
    p = tmp_path / "u.res"
    p.write_text("".join(lines), encoding="utf-8")
    run = _wrapper(load_run_file(p))
    qids = [str(k) for k in run]
    got = E._run_arrays_flat(run, qids)
    assert got is not None and list(got[1]) == sorted(got[1])
    _, want = _both(run)
    _assert_same(got, want)
