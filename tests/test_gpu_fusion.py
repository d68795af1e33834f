"""Parity of the HIP fusion kernel (qf_fuse) with the oracle — needs an MI355X.

Bit-exact is the bar: fused scores are compared as IEEE doubles, orders and
document ids exactly.
"""
import numpy as np
import pytest
import torch

from oracle import _loader as coracle
from oracle import ref_port
from tests.helpers import decode_fused, frames_from_rows, sorted_lists, first_seen_lists

pytestmark = pytest.mark.gpu

ALL = ["combsum", "combmnz", "rrf", "wcombsum", "wcombmnz", "wrrf"]


def _api():
    from qppfuse import fusion
    return fusion


@pytest.mark.parametrize("method", ["wcombsum", "wcombmnz", "wrrf"])
def test_weighted_api_matches_reference_golden(gpu, golden, method):
    fusion = _api()
    for case in golden["cases"]:
        frames = frames_from_rows(case["runs"], case["rankers"])
        fn = {"wcombsum": fusion.weighted_combsum, "wcombmnz": fusion.weighted_combmnz}.get(method)
        if fn is None:
            got = fusion.weighted_rrf(frames, case["qpp"], case["qpp_index"], k=case["rrf_k"])
        else:
            got = fn(frames, case["qpp"], case["qpp_index"])
        want = decode_fused(case["outputs"][method])
        assert sorted(got.keys()) == sorted(want.keys())
        for q in want:
            assert got[q] == want[q], (case["name"], method, q)


@pytest.mark.parametrize("method", ["combsum", "combmnz", "rrf"])
def test_unweighted_api_matches_port(gpu, golden, method):
    fusion = _api()
    for case in golden["cases"]:
        frames = frames_from_rows(case["runs"], case["rankers"])
        if case["name"] in ("unsorted_rankshift",):
            continue
        got = getattr(fusion, method)(frames)
        want = ref_port.ranx_fusion(frames, method, 60)
        for q in want:
            assert got[q] == want[q], (case["name"], method, q)


def test_write_runfile_bytes_match_reference(gpu, golden, tmp_path):
    fusion = _api()
    for case in golden["cases"]:
        frames = frames_from_rows(case["runs"], case["rankers"])
        res = fusion.fuse_many(frames, ["wcombsum", "wcombmnz", "wrrf"], case["qpp"],
                               case["qpp_index"], case["rrf_k"])
        for m, fused in res.items():
            p = tmp_path / f"{case['name']}_{m}.res"
            fusion.write_runfile(fused, str(p), f"{m}-tag")
            assert p.read_text() == case["runfiles"][m], (case["name"], m)


def _synthetic(Q, R, K, seed=11, p_shared=0.7):
    from qppfuse import engine
    off, docid, raw = engine.synth_runs(0, Q, R, K, seed=seed, p_shared=p_shared)
    norm, micro = engine.minmax_per_query(raw, off)
    return off, docid, raw, norm, micro


@pytest.mark.parametrize("shape", [(64, 3, 100), (200, 5, 1000), (40, 7, 1000), (300, 2, 37)])
def test_fuse_all_methods_bit_exact_vs_c_oracle(gpu, shape):
    from qppfuse import engine
    Q, R, K = shape
    off, docid, raw, norm, micro = _synthetic(Q, R, K)
    rng = np.random.default_rng(Q + R + K)
    w = torch.from_numpy(rng.random(Q * R).round(6)).to(gpu)
    out = engine.fuse(off, docid, micro, R, ALL, rrf_k=60, weights=w, max_entries=R * K)
    torch.cuda.synchronize()
    off_h = off.cpu().numpy()
    doc_h = docid.cpu().numpy().view(np.uint32)
    sc_h = micro.cpu().numpy().astype(np.float64) / 1e6
    w_h = w.cpu().numpy()
    ud = out.union_docid.cpu().numpy().view(np.uint32)
    uc = out.union_count.cpu().numpy()
    perm = _perm_np(out)
    fused = out.ranked_fused().cpu().numpy()
    assert (uc > 0).all()
    for m, name in enumerate(ALL):
        o_ud, o_uc, o_perm, o_fused = coracle.fuse(off_h, doc_h, sc_h, R, name, 60, weights=w_h)
        np.testing.assert_array_equal(uc, o_uc)
        for q in range(Q):
            b, n = off_h[q * R], uc[q]
            np.testing.assert_array_equal(ud[b:b + n], o_ud[b:b + n])
            np.testing.assert_array_equal(perm[m, b:b + n], o_perm[b:b + n], err_msg=f"{name} q{q}")
            assert fused[m, b:b + n].tobytes() == o_fused[b:b + n].tobytes(), (name, q)


def test_fuse_f64_scores_bit_exact(gpu):
    from qppfuse import engine
    Q, R, K = 50, 4, 250
    off, docid, raw, norm, micro = _synthetic(Q, R, K, seed=5)
    out = engine.fuse(off, docid, raw, R, ["combsum", "rrf", "combmnz"], max_entries=R * K)
    off_h, doc_h, raw_h = off.cpu().numpy(), docid.cpu().numpy().view(np.uint32), raw.cpu().numpy()
    uc = out.union_count.cpu().numpy()
    for m, name in enumerate(["combsum", "combmnz", "rrf"]):
        _, o_uc, o_perm, o_fused = coracle.fuse(off_h, doc_h, raw_h, R, name)
        f = out.ranked_fused().cpu().numpy()[m]
        p = _perm_np(out)[m]
        for q in range(Q):
            b, n = off_h[q * R], uc[q]
            assert f[b:b + n].tobytes() == o_fused[b:b + n].tobytes(), (name, q)
            np.testing.assert_array_equal(p[b:b + n], o_perm[b:b + n])


def test_bucket_sort_weight_extremes(gpu):
    """The join + bucket-sort path (1,500 entries per query) with the weights that stress
    its key: zero weights (hundreds of documents tied at the minimum), weights 1e-12 next
    to 1 (documents packed just above the minimum), negative weights and -0.0 (negative
    scores, signed zeros), 1e300 (a range near the f64 limit) — bit-exact vs the oracle."""
    from qppfuse import engine
    Q, R, K = 72, 5, 300
    off, docid, raw, norm, micro = _synthetic(Q, R, K, seed=21)
    rng = np.random.default_rng(21)
    # 1e-6 next to 1: the first count overflows a bucket, the finer recount does not;
    # 1e-12 next to 1: both overflow, the fallback pass sorts the pair
    cases = [[0.0, 0.0, 0.5, 0.3, 0.0], [1e-12, 1.0, 1.0, 1e-12, 1.0], [1e-6, 1.0, 0.5, 1e-6, 1.0],
             [-0.5, 0.2, -1.0, 0.0, 0.7], [-0.0] * 5, [1e300, 1e300, 1.0, 1.0, 1.0],
             list(rng.random(5))]
    w_h = np.array([cases[q % len(cases)] for q in range(Q)], np.float64).ravel()
    w = torch.from_numpy(w_h).to(gpu)
    out = engine.fuse(off, docid, micro, R, ALL, rrf_k=60, weights=w, max_entries=R * K)
    torch.cuda.synchronize()
    off_h = off.cpu().numpy()
    doc_h = docid.cpu().numpy().view(np.uint32)
    sc_h = micro.cpu().numpy().astype(np.float64) / 1e6
    uc = out.union_count.cpu().numpy()
    perm = _perm_np(out)
    fused = out.ranked_fused().cpu().numpy()
    assert (uc > 0).all()
    for m, name in enumerate(ALL):
        _, o_uc, o_perm, o_fused = coracle.fuse(off_h, doc_h, sc_h, R, name, 60, weights=w_h)
        np.testing.assert_array_equal(uc, o_uc)
        for q in range(Q):
            b, n = off_h[q * R], uc[q]
            np.testing.assert_array_equal(perm[m, b:b + n], o_perm[b:b + n], err_msg=f"{name} q{q}")
            assert fused[m, b:b + n].tobytes() == o_fused[b:b + n].tobytes(), (name, q)


def _csr(lists, device):
    off = np.cumsum([0] + [len(l[0]) for l in lists]).astype(np.int64)
    doc = np.concatenate([np.asarray(l[0], np.uint32) for l in lists] or [np.zeros(0, np.uint32)])
    sc = np.concatenate([np.asarray(l[1], np.float64) for l in lists] or [np.zeros(0)])
    t = lambda a: torch.from_numpy(a).to(device)
    return off, doc, sc, t(off), t(doc.view(np.int32)), t(sc)


@pytest.mark.parametrize("max_entries", [8, 2048, 20000])  # small join, LDS join, workspace join
def test_ranx_minmax_denominator_floor(gpu, max_entries):
    """ranx's min-max divides by max(max - min, 1e-9): a list whose range is below
    1e-9 is scaled by 1e-9 (not stretched to [0, 1]), a constant list gives 0."""
    from qppfuse import engine
    R = 3
    lists = [([1, 2, 3], [1.0 + 4e-10, 1.0 + 1e-10, 1.0]),   # range 4e-10 < 1e-9
             ([2, 4], [0.3, 0.3]),                           # constant
             ([3, 5, 1], [7.0, 5.0, 2.5])]                   # ordinary
    off, doc, sc, doff, ddoc, dsc = _csr(lists, gpu)
    out = engine.fuse(doff, ddoc, dsc, R, ["combsum", "combmnz", "rrf"],
                      max_entries=max_entries)
    uc = int(out.union_count[0])
    f = out.ranked_fused().cpu().numpy()
    p = _perm_np(out)
    for m, name in enumerate(["combsum", "combmnz", "rrf"]):
        _, o_uc, o_perm, o_fused = coracle.fuse(off, doc, sc, R, name)
        assert uc == o_uc[0] == 5
        assert f[m][:uc].tobytes() == o_fused[:uc].tobytes(), name
        np.testing.assert_array_equal(p[m][:uc], o_perm[:uc])
    ud = out.union_docid.cpu().numpy().view(np.uint32)
    got = dict(zip(ud[p[0][:uc].astype(np.int64)].tolist(), f[0][:uc].tolist()))
    want = {}
    for docs, scores in lists:  # the rule itself, in Python floats, runs in order
        lo, hi = min(scores), max(scores)
        den = max(hi - lo, 1e-9)
        for d, x in zip(docs, scores):
            want[d] = want.get(d, 0.0) + (x - lo) / den
    assert got == want


def test_edge_cases_empty_lists_ties_single(gpu):
    from qppfuse import engine
    R = 3
    lists = [  # q0: one retriever empty, ties everywhere
        ([1, 2, 3], [0.5, 0.5, 0.5]), ([], []), ([3, 2, 9], [1.0, 0.25, 0.25]),
        # q1: single entry
        ([7], [0.0]), ([], []), ([], []),
        # q2: identical lists in all retrievers
        ([4, 5, 6], [1.0, 0.5, 0.0]), ([4, 5, 6], [1.0, 0.5, 0.0]), ([4, 5, 6], [1.0, 0.5, 0.0]),
    ]
    off, doc, sc, doff, ddoc, dsc = _csr(lists, gpu)
    w = torch.tensor([0.3, 0.5, 0.2] * 3, dtype=torch.float64, device=gpu)
    out = engine.fuse(doff, ddoc, dsc, R, ALL, weights=w, max_entries=9)
    uc = out.union_count.cpu().numpy()
    for m, name in enumerate(ALL):
        o_ud, o_uc, o_perm, o_fused = coracle.fuse(off, doc, sc, R, name, weights=w.cpu().numpy())
        np.testing.assert_array_equal(uc, o_uc)
        np.testing.assert_array_equal(_perm_np(out)[m][:off[-1]][
            np.concatenate([np.arange(off[q * R], off[q * R] + uc[q]) for q in range(3)])],
            o_perm[np.concatenate([np.arange(off[q * R], off[q * R] + uc[q]) for q in range(3)])])
        f = out.ranked_fused().cpu().numpy()[m]
        for q in range(3):
            b, n = off[q * R], uc[q]
            assert f[b:b + n].tobytes() == o_fused[b:b + n].tobytes(), (name, q)


@pytest.mark.parametrize("n_entries", [1024, 1025, 5120, 5121, 7680, 7681, 10240, 10241, 65535,
                                       65536, 100_000])
def test_kernel_capacity_boundaries(gpu, n_entries):
    """Queries exactly at / just past each kernel configuration's capacity."""
    from qppfuse import engine
    R = 2
    rng = np.random.default_rng(n_entries)
    a = n_entries // 2
    docs = rng.choice(max(50_000, 2 * n_entries), size=n_entries, replace=False).astype(np.uint32)
    docs[a:a + a // 3] = docs[: a // 3]  # overlap between the two lists
    s1 = np.sort(rng.integers(0, 10**6, a))[::-1] / 1e6
    s2 = np.sort(rng.integers(0, 10**6, n_entries - a))[::-1] / 1e6
    lists = [(docs[:a], s1), (docs[a:], s2)]
    off, doc, sc, doff, ddoc, dsc = _csr(lists, gpu)
    out = engine.fuse(doff, ddoc, dsc, R, ["combsum", "rrf"], max_entries=n_entries)
    uc = out.union_count.cpu().numpy()
    for m, name in enumerate(["combsum", "rrf"]):
        _, o_uc, o_perm, o_fused = coracle.fuse(off, doc, sc, R, name)
        assert uc[0] == o_uc[0]
        n = uc[0]
        assert out.ranked_fused().cpu().numpy()[m][:n].tobytes() == o_fused[:n].tobytes()
        np.testing.assert_array_equal(_perm_np(out)[m][:n], o_perm[:n])


def test_too_big_and_unsorted_are_reported(gpu):
    from qppfuse import engine, _lib
    R = 1
    off, doc, sc, doff, ddoc, dsc = _csr([([1, 2, 3], [0.1, 0.9, 0.5])], gpu)
    out = engine.fuse(doff, ddoc, dsc, R, ["rrf"], max_entries=3)
    assert out.union_count.cpu().numpy()[0] == -2
    out = engine.fuse(doff, ddoc, dsc, R, ["wcombsum"], max_entries=3,
                      weights=torch.ones(1, dtype=torch.float64, device=gpu))
    assert out.union_count.cpu().numpy()[0] == 3  # weighted methods need no order
    with pytest.raises(_lib.QPPFuseError):
        engine.fuse(doff, ddoc, dsc, R, ["rrf"],
                    max_entries=_lib.max_entries_per_query_wide() + 1)
    small = engine.alloc_fuse_out(1, 3, _lib.RRF, gpu)  # uint16 perm: too narrow
    with pytest.raises(ValueError, match="uint32 perm"):
        engine.fuse(doff, ddoc, dsc, R, ["rrf"], max_entries=_lib.max_entries_per_query() + 1,
                    out=small)
    with pytest.raises(ValueError):
        engine.fuse(doff, ddoc, dsc, R, ["wrrf"], max_entries=3)  # no weights
    off, doc, sc, doff, ddoc, dsc = _csr([([1, 2, 1], [0.9, 0.5, 0.1]), ([4], [1.0])], gpu)
    out = engine.fuse(doff, ddoc, dsc, 2, ["combsum"], max_entries=4)
    assert out.union_count.cpu().numpy()[0] == -5  # duplicate docid inside one list


def _perm_np(out):
    """perm as numpy: uint16, or uint32 when the call took the wide entry points."""
    return out.perm.cpu().numpy().view(np.uint32 if out.wide else np.uint16)


def _sort_case(kind, n, rng):
    if kind == "wide_then_clustered":  # coarse window -> long equal-prefix runs -> fallback
        s = 1.0 + rng.integers(0, 1 << 20, n) * 2.0 ** -52
        s[: n // 50] = rng.choice([1e300, -1e300, 7.0, -3.0], n // 50)
    elif kind == "pairs":  # many short runs that only the low bits order
        base = rng.uniform(0, 1, n // 2)
        s = np.concatenate([base, base + rng.integers(1, 1 << 12, n // 2) * 2.0 ** -50])[:n]
        s = np.resize(s, n)
    elif kind == "huge_and_inf":  # score range overflows: the raw-key window path
        s = rng.uniform(-1, 1, n)
        s[: n // 10] = rng.choice([1.7e308, -1.7e308, np.inf, -np.inf, 0.0], n // 10)
    elif kind == "heavy_tie":  # > 128 equal scores above the minimum: a bucket overflows
        s = np.full(n, 0.5)
        s[: max(1, n // 20)] = rng.uniform(-1, 1, max(1, n // 20))
    elif kind == "zeros_and_ties":
        s = rng.choice([0.0, -0.0, 1.0, 0.5, 0.5 + 2.0 ** -40, -2.0 ** -1074], n)
    else:  # uniform
        s = rng.standard_normal(n) * 10.0 ** rng.integers(-30, 30, n)
    rng.shuffle(s)
    return s


@pytest.mark.parametrize("n", [1, 2, 63, 65, 300, 320, 321, 384, 385, 700, 2560, 2561, 2900,
                               3072, 3073, 7000, 7681, 10240, 10241, 40000, 70000])
@pytest.mark.parametrize("kind", ["wide_then_clustered", "pairs", "zeros_and_ties", "uniform",
                                  "huge_and_inf", "heavy_tie"])
def test_sort_is_stable_descending_on_adversarial_keys(gpu, kind, n):
    """One retriever, W-CombSUM with weight 1: the fused scores are the inputs, so the
    kernel's sort (LSD window + run fix-up + full-LSD fallback; above 10,240 the
    workspace bucket sort and its bitonic fallback, above 65,535 with the uint32 perm)
    is checked against a stable descending sort with -0.0 == +0.0 (Python's sorted(),
    src/fusion.py:488).  Up to 384 entries: the one-wave bucket sort, whose marked
    pairs (ties beyond a bucket, non-finite ranges) take the LSD sort in-workgroup."""
    from qppfuse import engine
    rng = np.random.default_rng(hash((kind, n)) & 0xFFFF)
    s = _sort_case(kind, n, rng)
    doc = np.arange(n, dtype=np.uint32) * 7 + 3
    off = np.array([0, n], np.int64)
    t = lambda a: torch.from_numpy(a).to(gpu)
    w = torch.ones(1, dtype=torch.float64, device=gpu)
    out = engine.fuse(t(off), t(doc.view(np.int32)), t(s), 1, ["wcombsum"], weights=w,
                      max_entries=n)
    assert int(out.union_count[0]) == n
    perm = _perm_np(out)[0][:n].astype(np.int64)
    fused = out.ranked_fused().cpu().numpy()[0][:n]
    want = np.argsort(-s, kind="stable")
    np.testing.assert_array_equal(perm, want)
    # defaultdict(float) accumulation: 0.0 + 1.0 * s, so -0.0 comes out as +0.0
    assert fused.tobytes() == (0.0 + s[want]).tobytes()


@pytest.mark.parametrize("k", [1, 10, 1000, 3000])
def test_fused_topk_compaction(gpu, k):
    """qf_fused_topk packs rank i < min(k, U_q) of every (query, method) row."""
    from qppfuse import engine
    Q, R, K = 6, 3, 700
    off, docid, raw = engine.synth_runs(0, Q, R, K, seed=3)
    _, micro = engine.minmax_per_query(raw, off, want_norm=False)
    ms = ["combsum", "rrf"]
    out = engine.fuse(off, docid, micro, R, ms, max_entries=R * K)
    d, s = engine.fused_topk(out, off, R, k)
    d, s = d.cpu().numpy().view(np.uint32), s.cpu().numpy()
    off_h, uc = off.cpu().numpy(), out.union_count.cpu().numpy()
    ud = out.union_docid.cpu().numpy().view(np.uint32)
    perm = _perm_np(out)
    fz = out.ranked_fused().cpu().numpy()
    for q in range(Q):
        b, n = off_h[q * R], min(k, uc[q])
        for m in range(len(ms)):
            np.testing.assert_array_equal(d[q, m, :n], ud[b + perm[m, b:b + n].astype(np.int64)])
            assert s[q, m, :n].tobytes() == fz[m, b:b + n].tobytes()
            assert (d[q, m, n:] == 0xFFFFFFFF).all() and np.isnan(s[q, m, n:]).all()


def test_grids_beyond_65536_workgroups(gpu):
    """Launches of more than 65,536 workgroups fold into a 2-D grid (a dispatch holds at
    most 2^32 - 1 work-items per dimension): the join (one workgroup per query), the six
    sorts, the min-max and the synthetic generator all run 2-D here, bit-exact."""
    from qppfuse import engine
    Q, R, K = 140_000, 2, 2
    off, docid, raw = engine.synth_runs(0, Q, R, K, seed=5)
    norm, micro = engine.minmax_per_query(raw, off)  # 70,000 workgroups
    rng = np.random.default_rng(9)
    w = torch.from_numpy(rng.random(Q * R).round(6)).to(gpu)
    out = engine.fuse(off, docid, micro, R, ALL, rrf_k=60, weights=w, max_entries=R * K)
    torch.cuda.synchronize()
    off_h = off.cpu().numpy()
    raw_h = raw.cpu().numpy()
    o_norm = coracle.minmax_per_query(raw_h, off_h)
    assert norm.cpu().numpy().tobytes() == o_norm.tobytes()
    sample = np.random.default_rng(2).choice(len(o_norm), 2000, replace=False)
    mh = micro.cpu().numpy()
    assert [f"{m // 10**6}.{m % 10**6:06d}" for m in mh[sample]] == \
        [f"{x:.6f}" for x in o_norm[sample]]
    doc_h = docid.cpu().numpy().view(np.uint32)
    sc_h = micro.cpu().numpy().astype(np.float64) / 1e6
    uc = out.union_count.cpu().numpy()
    ud = out.union_docid.cpu().numpy().view(np.uint32)
    perm = _perm_np(out)
    fused = out.ranked_fused().cpu().numpy()
    E = Q * R * K
    qb = np.repeat(off_h[0:-1:R][:Q], R * K)
    valid = (np.arange(E) - qb) < np.repeat(uc, R * K)
    for m, name in enumerate(ALL):
        o_ud, o_uc, o_perm, o_fused = coracle.fuse(off_h, doc_h, sc_h, R, name, 60,
                                                   weights=w.cpu().numpy())
        np.testing.assert_array_equal(uc, o_uc)
        np.testing.assert_array_equal(ud[valid], o_ud[valid])
        np.testing.assert_array_equal(perm[m][valid], o_perm[valid], err_msg=name)
        assert fused[m][valid].tobytes() == o_fused[valid].tobytes(), name


def test_bucket_sort_grid_beyond_65536_workgroups(gpu):
    """The bucket sort's (query, method) map runs the query groups in reverse: on a 2-D
    grid (more than 65,536 workgroups) the padding workgroups past the last pair must
    leave — 33,000 queries x 2 methods with 1,040 entries each (the join + bucket-sort
    path), checked against the oracle on a sample of queries."""
    from qppfuse import engine
    Q, R, K = 33_000, 2, 520
    ms = ["combsum", "rrf"]
    off, docid, raw = engine.synth_runs(0, Q, R, K, seed=13)
    _, micro = engine.minmax_per_query(raw, off, want_norm=False)
    out = engine.fuse(off, docid, micro, R, ms, rrf_k=60, max_entries=R * K)
    torch.cuda.synchronize()
    off_h = off.cpu().numpy()
    doc_h = docid.cpu().numpy().view(np.uint32)
    sc_h = micro.cpu().numpy().astype(np.float64) / 1e6
    uc = out.union_count.cpu().numpy()
    ud = out.union_docid.cpu().numpy().view(np.uint32)
    perm = _perm_np(out)
    fused = out.ranked_fused().cpu().numpy()
    qs = np.sort(np.random.default_rng(4).choice(Q, 300, replace=False))
    qs = np.concatenate([[0], qs, [Q - 1]])
    # the sampled queries as their own run set (queries are independent)
    lens = np.diff(off_h)
    sub_off = np.concatenate([[0], np.cumsum(lens.reshape(Q, R)[qs].ravel())])
    idx = np.concatenate([np.arange(off_h[q * R], off_h[q * R + R]) for q in qs])
    for m, name in enumerate(ms):
        o_ud, o_uc, o_perm, o_fused = coracle.fuse(sub_off, doc_h[idx], sc_h[idx], R, name, 60)
        np.testing.assert_array_equal(uc[qs], o_uc)
        for i, q in enumerate(qs):
            b, n, sb = off_h[q * R], uc[q], sub_off[i * R]
            np.testing.assert_array_equal(ud[b:b + n], o_ud[sb:sb + n])
            np.testing.assert_array_equal(perm[m][b:b + n], o_perm[sb:sb + n], err_msg=name)
            assert fused[m][b:b + n].tobytes() == o_fused[sb:sb + n].tobytes(), name


@pytest.mark.parametrize("kind", ["f64", "micro"])
def test_workspace_path_for_very_large_queries(gpu, kind):
    """Queries beyond the LDS join (more than 10,240 entries, up to 65,535) run the
    workspace join + bitonic sort (join_sort_xl_kernel); small queries of the same
    call still take the LDS kernels.  Every method bit-exact vs the oracle."""
    from qppfuse import engine
    R = 4
    rng = np.random.default_rng(11 if kind == "f64" else 12)
    sizes = [300, 5000, 0, 16383, 1, 2600]  # per-list K of each query
    lists, ranks = [], []
    for K in sizes:
        pool = rng.choice(1 << 30, size=max(1, 2 * K), replace=False).astype(np.uint32)
        for r in range(R):
            k = K if r != 2 else K // 2  # ragged lists
            docs = rng.choice(pool, size=k, replace=False)
            sc = np.sort(rng.integers(0, 3000 + r * 7919, k))[::-1] / 1e6  # ties
            lists.append((docs, sc))
            ranks.append(np.arange(1, k + 1, dtype=np.int32))
    off, doc, sc, doff, ddoc, dsc = _csr(lists, gpu)
    n_max = int(np.max(off[R::R] - off[0:-1:R]))
    assert n_max > 10240
    if kind == "micro":
        dsc = torch.from_numpy(np.rint(sc * 1e6).astype(np.int32)).to(gpu)
    rank = np.concatenate(ranks)
    w = rng.uniform(0.05, 1.0, len(sizes) * R)
    out = engine.fuse(doff, ddoc, dsc, R, ALL, rrf_k=60,
                      weights=torch.from_numpy(w).to(gpu),
                      rank=torch.from_numpy(rank).to(gpu), max_entries=n_max)
    uc = out.union_count.cpu().numpy()
    ud = out.union_docid.cpu().numpy().view(np.uint32)
    perm = _perm_np(out)
    fz = out.ranked_fused().cpu().numpy()
    for m, name in enumerate(ALL):
        o_ud, o_uc, o_perm, o_fused = coracle.fuse(off, doc, sc, R, name, 60, weights=w,
                                                   rank=rank)
        np.testing.assert_array_equal(uc, o_uc)
        for q in range(len(sizes)):
            b, n = off[q * R], uc[q]
            np.testing.assert_array_equal(ud[b:b + n], o_ud[b:b + n])
            np.testing.assert_array_equal(perm[m, b:b + n], o_perm[b:b + n], err_msg=f"{name} q{q}")
            assert fz[m, b:b + n].tobytes() == o_fused[b:b + n].tobytes(), (name, q)


@pytest.mark.parametrize("K", [6000, 12000, 50000])
def test_workspace_path_learned_ties_by_docid(gpu, K):
    """Learned fusion on a very large query: ties in docid order (the groupby's
    output order, src/fusion.py:443-446).  With two lists the Kahan sum equals
    the plain left-to-right sum, so the scores are W-CombSUM's.  K = 6000: a union
    of ~9,000 (the workspace join, then the LDS sort); K = 12000: ~18,000 (the
    workspace bucket sort, minimum's sub-buckets by docid); K = 50000: ~75,000 (the
    same with the uint32 perm)."""
    from qppfuse import engine
    R = 2
    rng = np.random.default_rng(5)
    pool = rng.choice(1 << 31, size=2 * K, replace=False).astype(np.uint32)
    lists = []
    for r in range(R):
        lists.append((rng.choice(pool, size=K, replace=False),
                      np.sort(rng.integers(0, 50, K))[::-1] / 1e6))
    off, doc, sc, doff, ddoc, dsc = _csr(lists, gpu)
    w = np.array([0.5, 0.25])
    out = engine.fuse(doff, ddoc, dsc, R, ["learned"], weights=torch.from_numpy(w).to(gpu),
                      max_entries=2 * K)
    o_ud, o_uc, o_perm, o_fused = coracle.fuse(off, doc, sc, R, "wcombsum", weights=w)
    n = int(out.union_count[0])
    assert n == o_uc[0]
    ud = out.union_docid.cpu().numpy().view(np.uint32)[:n]
    np.testing.assert_array_equal(ud, o_ud[:n])
    unsorted = np.empty(n)
    unsorted[o_perm[:n].astype(np.int64)] = o_fused[:n]
    want = np.lexsort((ud, -unsorted))
    perm = _perm_np(out)[0][:n].astype(np.int64)
    np.testing.assert_array_equal(perm, want)
    assert out.ranked_fused().cpu().numpy()[0][:n].tobytes() == unsorted[want].tobytes()


@pytest.mark.parametrize("R,K", [(17, 300), (32, 40), (20, 700)])
def test_more_than_16_runs_take_the_workspace_join(gpu, R, K):
    """More runs than the LDS join's 16-bit retriever masks: every query goes through
    the workspace join (32-bit masks), then the LDS sorts.  Every method bit-exact."""
    from qppfuse import engine
    rng = np.random.default_rng(R * 1000 + K)
    sizes = [K, 0, K // 3, 1, K]
    lists, ranks = [], []
    for k0 in sizes:
        pool = rng.choice(1 << 30, size=max(1, 3 * k0), replace=False).astype(np.uint32)
        for r in range(R):
            k = k0 if r % 5 else k0 // 2  # ragged
            docs = rng.choice(pool, size=k, replace=False)
            lists.append((docs, np.sort(rng.integers(0, 2000, k))[::-1] / 1e6))
            ranks.append(np.arange(1, k + 1, dtype=np.int32))
    off, doc, sc, doff, ddoc, dsc = _csr(lists, gpu)
    n_max = int(np.max(off[R::R] - off[0:-1:R]))
    rank = np.concatenate(ranks)
    w = rng.uniform(0.05, 1.0, len(sizes) * R)
    out = engine.fuse(doff, ddoc, dsc, R, ALL, rrf_k=60, weights=torch.from_numpy(w).to(gpu),
                      rank=torch.from_numpy(rank).to(gpu), max_entries=n_max)
    uc = out.union_count.cpu().numpy()
    ud = out.union_docid.cpu().numpy().view(np.uint32)
    perm = _perm_np(out)
    fz = out.ranked_fused().cpu().numpy()
    for m, name in enumerate(ALL):
        o_ud, o_uc, o_perm, o_fused = coracle.fuse(off, doc, sc, R, name, 60, weights=w,
                                                   rank=rank)
        np.testing.assert_array_equal(uc, o_uc)
        for q in range(len(sizes)):
            b, n = off[q * R], uc[q]
            np.testing.assert_array_equal(ud[b:b + n], o_ud[b:b + n])
            np.testing.assert_array_equal(perm[m, b:b + n], o_perm[b:b + n], err_msg=f"{name} q{q}")
            assert fz[m, b:b + n].tobytes() == o_fused[b:b + n].tobytes(), (name, q)


def test_workspace_join_reports_queries_beyond_max_entries(gpu):
    """17 runs (the workspace join for every query) with one query larger than the
    max_entries the caller passes: that query reports QF_QSTATUS_TOOBIG instead of
    leaving its union_count unwritten; the others are fused as usual."""
    from qppfuse import engine, _lib
    R = 17
    rng = np.random.default_rng(17)
    lists = []
    for q, k in enumerate((4, 9, 3)):
        for r in range(R):
            docs = rng.choice(1000, size=k, replace=False).astype(np.uint32)
            lists.append((docs, np.sort(rng.integers(0, 10**6, k))[::-1] / 1e6))
    off, doc, sc, doff, ddoc, dsc = _csr(lists, gpu)
    out = engine.fuse(doff, ddoc, dsc, R, ["combsum", "rrf"], max_entries=4 * R)
    uc = out.union_count.cpu().numpy()
    assert uc[1] == _lib.QF_QSTATUS_TOOBIG
    o_ud, o_uc, o_perm, o_fused = coracle.fuse(off, doc, sc, R, "combsum", 60)
    for q in (0, 2):
        b, n = off[q * R], uc[q]
        assert n == o_uc[q] > 0
        assert out.ranked_fused().cpu().numpy()[0][b:b + n].tobytes() == o_fused[b:b + n].tobytes()


def test_more_than_32_runs_are_rejected(gpu):
    from qppfuse import engine
    R = 33
    off, doc, sc, doff, ddoc, dsc = _csr([([r + 1], [1.0]) for r in range(R)], gpu)
    with pytest.raises(ValueError, match="n_retrievers"):  # QF_EINVAL
        engine.fuse(doff, ddoc, dsc, R, ["combsum"], max_entries=R)


def test_api_with_18_rankers_matches_port(gpu):
    """The reference API with more rankers than the LDS join holds (18): every method
    through qppfuse.fusion, equal to the row-by-row port (weighted: the reference's
    loops; unweighted: ranx semantics)."""
    import pandas as pd
    fusion = _api()
    rng = np.random.default_rng(18)
    rankers = [f"R{i:02d}" for i in range(18)]
    frames, qpp = {}, {}
    for r in rankers:
        rows = []
        for q in range(6):
            k = int(rng.integers(0, 40))
            docs = rng.choice(120, size=k, replace=False)
            sc = np.sort(rng.integers(0, 10**6, k))[::-1] / 1e6
            rows += [(f"test{q}", f"doc{d}", i + 1, s) for i, (d, s) in enumerate(zip(docs, sc))]
        df = pd.DataFrame(rows, columns=["qid", "docno", "rank", "score"])
        df.insert(1, "iter", "Q0")
        df["runid"] = r
        frames[r] = df
    for q in range(6):
        qpp[f"test{q}"] = {r: list(rng.uniform(0, 1, 13)) for r in rankers}
    for name, fn in [("wcombsum", fusion.weighted_combsum), ("wcombmnz", fusion.weighted_combmnz)]:
        got = fn(frames, qpp, 5)
        want = ref_port.weighted_fusion(frames, qpp, 5, name)
        for q in want:
            assert got[q] == want[q], (name, q)
    got = fusion.weighted_rrf(frames, qpp, -1, k=60)
    want = ref_port.weighted_fusion(frames, qpp, -1, "wrrf", 60)
    for q in want:
        assert got[q] == want[q], ("wrrf", q)
    for method in ["combsum", "combmnz", "rrf"]:
        got = getattr(fusion, method)(frames)
        want = ref_port.ranx_fusion(frames, method, 60)
        for q in want:
            assert got[q] == want[q], (method, q)


@pytest.mark.parametrize("methods", [["combmnz"], ["combmnz", "rrf"], ["wcombsum", "wcombmnz"],
                                     ["combsum", "combmnz", "wcombmnz"],
                                     ["combsum", "wcombsum", "wcombmnz", "wrrf"]])
def test_method_subsets_bit_exact(gpu, methods):
    """Subsets of the six methods (output slots shift with the mask; CombMNZ with and
    without its CombSUM) bit-exact vs the oracle on the join + bucket-sort path (5 x
    1,000 entries)."""
    from qppfuse import engine
    Q, R, K = 96, 5, 1000
    off, docid, raw, norm, micro = _synthetic(Q, R, K, seed=31)
    rng = np.random.default_rng(31)
    w = torch.from_numpy(rng.random(Q * R).round(6)).to(gpu)
    out = engine.fuse(off, docid, micro, R, methods, rrf_k=60, weights=w, max_entries=R * K)
    torch.cuda.synchronize()
    off_h = off.cpu().numpy()
    doc_h = docid.cpu().numpy().view(np.uint32)
    sc_h = micro.cpu().numpy().astype(np.float64) / 1e6
    uc = out.union_count.cpu().numpy()
    perm = _perm_np(out)
    fused = out.ranked_fused().cpu().numpy()
    slot = {m: i for i, m in enumerate(sorted(methods, key=ALL.index))}
    for name in methods:
        _, o_uc, o_perm, o_fused = coracle.fuse(off_h, doc_h, sc_h, R, name, 60,
                                                weights=w.cpu().numpy())
        np.testing.assert_array_equal(uc, o_uc)
        m = slot[name]
        for q in range(Q):
            b, n = off_h[q * R], uc[q]
            np.testing.assert_array_equal(perm[m, b:b + n], o_perm[b:b + n], err_msg=f"{name} q{q}")
            assert fused[m, b:b + n].tobytes() == o_fused[b:b + n].tobytes(), (name, q)


@pytest.mark.parametrize("n", [700, 2561, 3072, 3073, 5120])
@pytest.mark.parametrize("overlap", [1.0, 0.02])
@pytest.mark.parametrize("kind", ["wide_then_clustered", "pairs", "zeros_and_ties", "uniform",
                                  "huge_and_inf"])
def test_two_runs_on_adversarial_keys(gpu, kind, overlap, n):
    """W-CombSUM + W-CombMNZ over two runs sharing a fraction of their documents, on the
    adversarial keys: the join + bucket-sort path, its fallback pass (a bucket above
    128 items, a non-finite range) and, for unions above 3,072 (up to 10,140),
    fuse_large_kernel — bit-exact vs the oracle."""
    from qppfuse import engine
    rng = np.random.default_rng(hash((kind, n, overlap)) & 0xFFFF)
    s1, s2 = _sort_case(kind, n, rng), _sort_case(kind, n, rng)
    if kind == "huge_and_inf":  # no inf - inf = NaN in a shared document's sum
        s1, s2 = np.abs(s1), np.abs(s2)
    d1 = np.arange(n, dtype=np.uint32) * 7 + 3
    shared = int(n * overlap)
    d2 = np.concatenate([d1[:shared][rng.permutation(shared)],
                         np.arange(n - shared, dtype=np.uint32) * 7 + 5])
    off = np.array([0, n, 2 * n], np.int64)
    doc = np.concatenate([d1, d2])
    sc = np.concatenate([s1, s2])
    t = lambda a: torch.from_numpy(a).to(gpu)
    w_h = np.array([1.0, 0.75])
    ms = ["wcombsum", "wcombmnz"]
    out = engine.fuse(t(off), t(doc.view(np.int32)), t(sc), 2, ms, weights=t(w_h),
                      max_entries=2 * n)
    uc = int(out.union_count[0])
    perm = _perm_np(out)
    fused = out.ranked_fused().cpu().numpy()
    for m, name in enumerate(ms):
        _, o_uc, o_perm, o_fused = coracle.fuse(off, doc, sc, 2, name, 60, weights=w_h)
        assert uc == o_uc[0] == 2 * n - shared
        np.testing.assert_array_equal(perm[m][:uc], o_perm[:uc], err_msg=name)
        assert fused[m][:uc].tobytes() == o_fused[:uc].tobytes(), name


def _wide_case(rng, sizes, R, pool_factor=2):
    lists, ranks = [], []
    for K in sizes:
        pool = rng.choice(1 << 30, size=max(1, pool_factor * K), replace=False).astype(np.uint32)
        for r in range(R):
            k = K if r != 2 else K // 2  # ragged lists
            docs = rng.choice(pool, size=k, replace=False)
            lists.append((docs, np.sort(rng.integers(0, 400_000 + r * 7919, k))[::-1] / 1e6))
            ranks.append(np.arange(1, k + 1, dtype=np.int32))
    return lists, np.concatenate(ranks)


@pytest.mark.parametrize("kind", ["f64", "micro"])
def test_wide_perm_queries_beyond_65535_entries(gpu, kind):
    """qf_fuse_wide: a query of 100,000+ entries whose union exceeds 65,535 documents
    (u needs 32 bits) next to small, mid-size and 40,000-entry queries in the same
    call — every path writes the uint32 perm — bit-exact vs the oracle for every
    method; qf_fused_topk_wide packs the same ranks."""
    from qppfuse import engine, _lib
    R = 4
    rng = np.random.default_rng(21 if kind == "f64" else 22)
    sizes = [300, 29_000, 0, 2600, 11_000, 1]  # per-list K: 101,500 entries in query 1
    lists, rank = _wide_case(rng, sizes, R, pool_factor=5)
    off, doc, sc, doff, ddoc, dsc = _csr(lists, gpu)
    n_max = int(np.max(off[R::R] - off[0:-1:R]))
    assert n_max > _lib.max_entries_per_query()
    if kind == "micro":
        dsc = torch.from_numpy(np.rint(sc * 1e6).astype(np.int32)).to(gpu)
    w = rng.uniform(0.05, 1.0, len(sizes) * R)
    out = engine.fuse(doff, ddoc, dsc, R, ALL, rrf_k=60, weights=torch.from_numpy(w).to(gpu),
                      rank=torch.from_numpy(rank).to(gpu), max_entries=n_max)
    assert out.wide
    uc = out.union_count.cpu().numpy()
    assert uc[1] > 65535
    ud = out.union_docid.cpu().numpy().view(np.uint32)
    perm = _perm_np(out)
    fz = out.ranked_fused().cpu().numpy()
    for m, name in enumerate(ALL):
        o_ud, o_uc, o_perm, o_fused = coracle.fuse(off, doc, sc, R, name, 60, weights=w,
                                                   rank=rank)
        np.testing.assert_array_equal(uc, o_uc)
        for q in range(len(sizes)):
            b, n = off[q * R], uc[q]
            np.testing.assert_array_equal(ud[b:b + n], o_ud[b:b + n])
            np.testing.assert_array_equal(perm[m, b:b + n], o_perm[b:b + n], err_msg=f"{name} q{q}")
            assert fz[m, b:b + n].tobytes() == o_fused[b:b + n].tobytes(), (name, q)
    k = 70_000
    d, s = engine.fused_topk(out, doff, R, k)
    d, s = d.cpu().numpy().view(np.uint32), s.cpu().numpy()
    for q in range(len(sizes)):
        b, n = off[q * R], min(k, uc[q])
        for m in range(len(ALL)):
            np.testing.assert_array_equal(d[q, m, :n], ud[b + perm[m, b:b + n].astype(np.int64)])
            assert s[q, m, :n].tobytes() == fz[m, b:b + n].tobytes()


def test_wide_api_fuse_and_write_runfile(gpu, tmp_path):
    """The reference's API over a query of 3 x 40,000 entries (union ~84,000):
    fuse_many takes the wide path; the FusedRun's ranked lists and write_runfile's
    bytes equal the restated reference's (oracle/ref_port.py) on the same runs."""
    import pandas as pd
    rng = np.random.default_rng(31)
    K = 40_000
    pool = np.array([f"d{i:07d}" for i in rng.choice(10**7, size=3 * K, replace=False)])
    frames = {}
    for name in ("bm25", "splade", "tct"):
        docs = rng.choice(pool, size=K, replace=False)
        sc = np.sort(rng.integers(0, 10**6, K))[::-1] / 1e6
        frames[name] = pd.DataFrame({"qid": "q1", "iter": "Q0", "docno": docs,
                                     "rank": np.arange(1, K + 1), "score": sc, "runid": name})
    fusion = _api()
    got = fusion.fuse_many(frames, ["combsum", "rrf"])
    for m in ("combsum", "rrf"):
        want = ref_port.fuse(frames, m)
        assert len(want["q1"]) > 65535
        assert got[m]["q1"] == want["q1"], m
        path = tmp_path / f"{m}.res"
        fusion.write_runfile(got[m], str(path), m)
        assert path.read_text() == ref_port.runfile_text(want, m), m
    # the IR evaluation of the wide FusedRun (its lists go over in rank order)
    from qppfuse.evaluation import IREvaluator
    ev = IREvaluator(["nDCG@10", "RR@10", "R@100", "P@10"])
    ranked = [d for d, _ in got["rrf"]["q1"]]
    qrels = {"q1": {ranked[i]: 1 + i % 2 for i in (0, 7, 500, 70_000)} | {"dx": 1}}
    assert ev.evaluate(got["rrf"], qrels, per_query=True) == \
        ev.evaluate({"q1": got["rrf"]["q1"]}, qrels, per_query=True)


@pytest.mark.parametrize("share", ["full", "one"])
def test_caller_owned_workspace(gpu, share):
    """qf_fuse_ws: the workspace kernel in the caller's buffer (the full size
    qf_fuse_workspace_bytes names, or one workgroup's share: fewer workgroups),
    100,000-entry and small queries in one call, bit-exact vs the oracle and
    identical to the stream-ordered allocation's outputs; reused twice."""
    from qppfuse import engine
    R = 4
    rng = np.random.default_rng(44)
    sizes = [25000, 300, 16383, 0, 2600]
    lists = []
    for K in sizes:
        pool = rng.choice(1 << 30, size=max(1, 2 * K), replace=False).astype(np.uint32)
        for r in range(R):
            k = K if r != 1 else K // 3
            docs = rng.choice(pool, size=k, replace=False)
            lists.append((docs, np.sort(rng.integers(0, 5000 + r * 7919, k))[::-1] / 1e6))
    off, doc, sc, doff, ddoc, dsc = _csr(lists, gpu)
    n_max = int(np.max(off[R::R] - off[0:-1:R]))
    assert n_max > 65535  # the wide perm
    w = rng.uniform(0.05, 1.0, len(sizes) * R)
    wd = torch.from_numpy(w).to(gpu)
    full = engine.workspace_bytes(len(sizes), R, n_max, ALL)
    one = engine.workspace_bytes(1, R, n_max, ALL)
    assert full >= one > 0
    ws = torch.empty(full if share == "full" else one, dtype=torch.uint8, device=gpu)
    ref = engine.fuse(doff, ddoc, dsc, R, ALL, 60, weights=wd, max_entries=n_max)
    rc = ref.union_count.cpu().numpy()
    for _ in range(2):
        out = engine.fuse(doff, ddoc, dsc, R, ALL, 60, weights=wd, max_entries=n_max,
                          workspace=ws)
        torch.cuda.synchronize()
        assert torch.equal(out.union_count, ref.union_count)
        for q in range(len(sizes)):  # every query's slots (the rest is never written)
            b, n = int(off[q * R]), int(rc[q])
            assert torch.equal(out.union_docid[b:b + n], ref.union_docid[b:b + n])
            assert torch.equal(out.perm[:, b:b + n], ref.perm[:, b:b + n])
            assert torch.equal(out.fused[:, b:b + n].view(torch.int64),
                               ref.fused[:, b:b + n].view(torch.int64))
    uc = out.union_count.cpu().numpy()
    perm = _perm_np(out)
    fz = out.ranked_fused().cpu().numpy()
    for m, name in enumerate(ALL):
        _, o_uc, o_perm, o_fused = coracle.fuse(off, doc, sc, R, name, 60, weights=w)
        np.testing.assert_array_equal(uc, o_uc)
        for q in range(len(sizes)):
            b, n = off[q * R], uc[q]
            np.testing.assert_array_equal(perm[m, b:b + n], o_perm[b:b + n], err_msg=name)
            assert fz[m, b:b + n].tobytes() == o_fused[b:b + n].tobytes(), (name, q)


@pytest.mark.parametrize("R,K", [(5, 40), (5, 160), (5, 400), (20, 50)])
@pytest.mark.parametrize("mode,qidx", [("minmax", 5), ("minmax", -1), ("minmax", 0),
                                       ("zscore", 5), ("zscore", -1)])
def test_fuse_qpp_weights_in_kernel_equal_normalize_then_fuse(gpu, mode, qidx, R, K):
    """qf_fuse_qpp (the W-* weights computed in the join from the raw QPP predictors
    and their column statistics) == qf_qpp_normalize's weights fed to qf_fuse, bit
    for bit: union sizes, every method's fused scores and perm; absent lists (weight
    from a 0.0 value), a constant QPP column.  Every join that computes list_weight:
    the one-wave join (R*K <= 320), the 256-thread one (<= 1,024), the 512-thread one,
    and the workspace kernel's (R = 20 > 16 runs)."""
    from qppfuse import engine
    Q = 300
    off, docid, raw = engine.synth_runs(11, Q, R, K)
    lens = torch.diff(off).cpu().numpy()
    # empty some lists: rebuild the run set without their entries
    drop = np.zeros(Q * R, bool)
    drop[[3, 17, 18, 250]] = True
    keep = np.repeat(~drop, lens)
    off_h = off.cpu().numpy()
    n2 = np.where(drop, 0, lens)
    off2 = torch.from_numpy(np.concatenate([[0], np.cumsum(n2)]).astype(np.int64)).to(gpu)
    kt = torch.from_numpy(keep).to(gpu)
    docid2, raw2 = docid[kt].contiguous(), raw[kt].contiguous()
    _, micro = engine.minmax_per_query(raw2, off2, want_norm=False)
    nt = torch.full((Q,), 3, dtype=torch.int32, device=gpu)
    tf = torch.rand((Q, 2), dtype=torch.float64, device=gpu,
                    generator=torch.Generator(gpu).manual_seed(2))
    qraw = engine.qpp_raw(raw2, off2, R, 100, nt, tf)
    qraw[:, 7] = 0.75  # a constant column
    stats = (engine.qpp_colminmax if mode == "minmax" else engine.qpp_colmeanstd)(qraw, off2, R)
    w = engine.qpp_normalize(qraw, stats, off2, R, mode, qidx, want_micro=False)["weights"]
    M = ["combsum", "combmnz", "rrf", "wcombsum", "wcombmnz", "wrrf"]
    a = engine.fuse(off2, docid2, micro, R, M, 60, weights=w, max_entries=R * K)
    b = engine.fuse(off2, docid2, micro, R, M, 60, max_entries=R * K,
                    qpp=(qraw, stats, mode, qidx))
    assert torch.equal(a.union_count, b.union_count)
    uc = a.union_count.cpu().numpy()
    fa, fb = a.fused.cpu().numpy(), b.fused.cpu().numpy()
    pa, pb = a.perm.cpu().numpy(), b.perm.cpu().numpy()
    lo = off2.cpu().numpy()
    for q in range(Q):
        s, u = int(lo[q * R]), int(uc[q])
        assert fa[:, s:s + u].tobytes() == fb[:, s:s + u].tobytes(), q
        assert np.array_equal(pa[:, s:s + u], pb[:, s:s + u]), q
    # qf_fuse_qpp_micro: the same fusion plus every list's 13 ".qpp" micro-units,
    # written by the join (each join configuration) — qpp_normalize's, bit for bit
    qm = torch.full((Q * R * 13,), -7, dtype=torch.int64, device=gpu)
    if R > 16:  # the workspace join (more runs than the LDS join's masks) writes none
        with pytest.raises(Exception):
            engine.fuse(off2, docid2, micro, R, M, 60, max_entries=R * K,
                        qpp=(qraw, stats, mode, qidx), qpp_micro_out=qm)
        return
    c = engine.fuse(off2, docid2, micro, R, M, 60, max_entries=R * K,
                    qpp=(qraw, stats, mode, qidx), qpp_micro_out=qm)
    want = engine.qpp_normalize(qraw, stats, off2, R, mode, qidx)["micro"]
    assert torch.equal(qm, want.reshape(-1).to(torch.int64))
    assert torch.equal(c.union_count, b.union_count)
    fc, pc = c.fused.cpu().numpy(), c.perm.cpu().numpy()
    for q in range(Q):
        s, u = int(lo[q * R]), int(uc[q])
        assert fc[:, s:s + u].tobytes() == fb[:, s:s + u].tobytes(), q
        assert np.array_equal(pc[:, s:s + u], pb[:, s:s + u]), q


@pytest.mark.parametrize("max_entries", [2000, 12000])
def test_fuse_qpp_micro_for_queries_past_the_lds_join(gpu, max_entries):
    """qf_fuse_qpp_micro writes the .qpp micro-units of a query the LDS join does not
    take: reported QF_QSTATUS_TOOBIG (max_entries 2,000 below its 2,400 x 5 entries) or
    joined by the workspace kernel (max_entries 12,000 > 10,240) — the values come from
    the LDS join's early exit either way."""
    from qppfuse import engine
    Q, R, K = 24, 5, 2400
    off, docid, raw = engine.synth_runs(5, Q, R, K)
    _, micro = engine.minmax_per_query(raw, off, want_norm=False)
    nt = torch.full((Q,), 4, dtype=torch.int32, device=gpu)
    tf = torch.rand((Q, 2), dtype=torch.float64, device=gpu,
                    generator=torch.Generator(gpu).manual_seed(3))
    qraw = engine.qpp_raw(raw, off, R, 100, nt, tf)
    stats = engine.qpp_colminmax(qraw, off, R)
    qm = torch.full((Q * R * 13,), -7, dtype=torch.int64, device=gpu)
    out = engine.fuse(off, docid, micro, R, ["wcombsum", "rrf"], 60, max_entries=max_entries,
                      qpp=(qraw, stats, "minmax", 5), qpp_micro_out=qm)
    want = engine.qpp_normalize(qraw, stats, off, R, "minmax", 5)["micro"]
    assert torch.equal(qm, want.reshape(-1).to(torch.int64))
    from qppfuse import _lib
    uc = out.union_count.cpu().numpy()
    if max_entries < R * K:
        assert (uc == _lib.QF_QSTATUS_TOOBIG).all()
    else:
        assert (uc > 0).all()


def _bs_key2(smin, smax, shift=8, minbase=3840):
    """Python restatement of qf_fuse.hip's bs_key2 (the bucket key's constants)."""
    import math
    import struct
    hi = lambda x: struct.unpack("<Q", struct.pack("<d", x))[0] >> 32
    rng = smax - smin
    delta = math.ldexp(rng, -shift)
    if not (math.isfinite(rng) and delta > 0.0):
        return None
    c = delta - smin
    cform = math.isfinite(c) and (smin + c) >= 0.5 * delta
    xmin = smin + c if cform else delta
    xmax = smax + c if cform else rng + delta
    if not math.isfinite(xmax):
        return None
    b0, top = hi(xmin), hi(xmax)
    span = (top - b0 + 1) & 0xFFFFFFFF
    scale = 0xFFFFFFFF if span <= minbase else int(minbase * 4294967296.0 / span) - 1
    return (c if cform else delta), (scale << 32) | (int(cform) << 31) | top


@pytest.mark.parametrize("methods", [ALL, ["combsum", "rrf"], ["wcombsum"], ["rrf"],
                                     ["combsum", "wcombsum"]])
def test_join_leaves_the_sort_key_constants(gpu, methods):
    """Round 5: the join reduces every method slot's min / max over the query's documents
    (register exchanges across the wave, then across waves) and leaves the bucket sort's
    key constants at fused[slot][base + U .. + 4) when the query has 4 spare slots:
    [min, max, c, top | cform << 31 | scale << 32] — exactly the values' extremes (-0.0
    folded) and bs_key2's constants; a run-time method set (no compile-time slots)
    leaves w3 = 0 (the sort computes them).  The fused outputs are checked elsewhere."""
    from qppfuse import engine
    Q, R, K = 48, 5, 1000
    off, docid, raw, norm, micro = _synthetic(Q, R, K, seed=5)
    rng = np.random.default_rng(3)
    w = torch.from_numpy(rng.random(Q * R).round(6)).to(gpu)
    w[:R] = 0.0  # query 0: zero weights, outside the sums' division-free fast path
    out = engine.fuse(off, docid, micro, R, methods, rrf_k=60, weights=w, max_entries=R * K)
    torch.cuda.synchronize()
    off_h = off.cpu().numpy()
    uc = out.union_count.cpu().numpy()
    fz = out.fused.cpu().numpy()
    compile_time = methods in (ALL, ["combsum", "rrf"], ["wcombsum"], ["rrf"])
    checked = 0
    for q in range(Q):
        b, n, N = off_h[q * R], uc[q], off_h[q * R + R] - off_h[q * R]
        if N - n < 4:
            continue
        for m in range(len(methods)):
            vals = fz[m, b:b + n]
            info = fz[m, b + n:b + n + 4]
            w3 = int(info[3:4].view(np.uint64)[0])
            if not compile_time or q == 0:  # the sort computes the constants itself
                assert w3 == 0, (q, m)
                continue
            smin, smax = float(vals.min()) + 0.0, float(vals.max()) + 0.0
            assert info[0].tobytes() == np.float64(smin).tobytes(), (q, m)
            assert info[1].tobytes() == np.float64(smax).tobytes(), (q, m)
            k = _bs_key2(smin, smax)
            if k is None:
                assert w3 == 0xFFFFFFFFFFFFFFFF, (q, m)
            else:
                assert info[2].tobytes() == np.float64(k[0]).tobytes(), (q, m)
                assert w3 == k[1], (q, m, hex(w3), hex(k[1]))
            checked += 1
    assert checked >= (Q - 1) * len(methods) if compile_time else True


@pytest.mark.parametrize("max_entries", [2048, 3072])
def test_understated_max_entries_still_sorted(gpu, max_entries):
    """the LDS join holds queries of up to 5,120 entries whatever
    max_entries says, so a caller whose max_entries (1,025-3,072) understates a query
    gets a union above 3,072 that the 512-thread bucket sort leaves and the 1,024-thread
    configuration (launched only for max_entries > 3,072) never sees.  The fallback
    pass now takes any such pair (FuseParams.fast_reach): every query bit-exact vs the
    C oracle, none left with an uninitialised perm."""
    import bench
    from qppfuse import engine
    Q, R, K = 16, 5, 900  # N = 4,500 entries per query, unions ~3,600 (SURVEY 8(d) data)
    qo, qd = bench.nq_qrels()
    off, docid, raw = engine.synth_runs_nq(0, Q, R, K, qo, qd)
    _, micro = engine.minmax_per_query(raw, off, want_norm=False)
    w = torch.from_numpy(np.random.default_rng(5).random(Q * R).round(6)).to(gpu)
    out = engine.fuse(off, docid, micro, R, ALL, rrf_k=60, weights=w, max_entries=max_entries)
    torch.cuda.synchronize()
    off_h = off.cpu().numpy()
    doc_h = docid.cpu().numpy().view(np.uint32)
    sc_h = micro.cpu().numpy().astype(np.float64) / 1e6
    uc = out.union_count.cpu().numpy()
    assert (uc > 3072).all(), uc
    perm = _perm_np(out)
    fused = out.ranked_fused().cpu().numpy()
    for m, name in enumerate(ALL):
        _, o_uc, o_perm, o_fused = coracle.fuse(off_h, doc_h, sc_h, R, name, 60,
                                                weights=w.cpu().numpy())
        assert np.array_equal(uc, o_uc), name
        for q in range(Q):
            b, n = off_h[q * R], uc[q]
            assert np.array_equal(perm[m, b:b + n], o_perm[b:b + n]), (name, q)
            assert fused[m, b:b + n].tobytes() == o_fused[b:b + n].tobytes(), (name, q)
