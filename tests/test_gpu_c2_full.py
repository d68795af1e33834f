"""The headline configuration pinned directly — needs an MI355X.

BASELINE.json's metric is quoted on C2: 3,452 queries x 5 retrievers x top-1,000,
min-max + the QPP predictors + all six fusions, full sorted lists.  bench.py's default
step runs it on SURVEY §8(d)'s generator (qf_synth_runs_nq, seed 20251212, the NQ
test qrels planted), whose unions (3,856-4,148 documents) take the large-union sort.
Here the WHOLE batch goes through the step's own calls and every query of every
method is compared with the C restatement of src/fusion.py (oracle/fusion_oracle.c):
  * union_count and union_docid (first-seen order, src/fusion.py:264-279),
  * perm (score descending, ties in first-seen order: src/fusion.py:475,488),
  * the fused scores (first-seen order and ranked), bit for bit,
  * the W-* weights: RSD (qpp_index 5, the reference's default) computed inside the
    fusion from the raw predictors (qf_fuse_qpp), fed to the oracle as the weights
    qf_qpp_normalize gives (the same bits, tests/test_gpu_qpp_scale.py).
The step's `.qpp` output — all 13 columns' "%.6f" micro-units, written by the join
(qf_fuse_qpp_micro) — is checked against qf_qpp_normalize and against Python's own
"%.6f" of the C restatement's normalised columns (src/qpp.py:324-334).
A second case runs the same batch through max_entries 7,680 (the join_kernel +
bsort_fast_kernel path of larger queries) and requires identical outputs.
"""
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from oracle import _loader as coracle

pytestmark = pytest.mark.gpu

Q, R, K = 3452, 5, 1000
METHODS = ["combsum", "combmnz", "rrf", "wcombsum", "wcombmnz", "wrrf"]


@pytest.fixture(scope="module")
def c2(gpu):
    import bench
    from qppfuse import engine as e
    off, docid, raw = bench.gen_runs(SimpleNamespace(generator="nq"), 0, Q, R, K)
    nt_h, tf_h = bench.text_inputs(0, Q)
    nt, tf = torch.from_numpy(nt_h).to(gpu), torch.from_numpy(tf_h).to(gpu)
    qraw = e.qpp_raw(raw, off, R, 100, nt, tf)
    micro = torch.empty(raw.numel(), dtype=torch.int32, device=gpu)
    mm = torch.empty(2 * R * 13, dtype=torch.float64, device=gpu)
    e.minmax_colminmax(raw, off, R, qraw, micro_out=micro, mm_out=mm)
    qmicro = torch.empty(Q * R * 13, dtype=torch.int64, device=gpu)
    out = e.fuse(off, docid, micro, R, METHODS, 60, max_entries=R * K,
                 qpp=(qraw, mm, "minmax", 5), qpp_micro_out=qmicro)
    torch.cuda.synchronize()
    return SimpleNamespace(off=off, docid=docid, raw=raw, micro=micro, qraw=qraw, mm=mm,
                           qmicro=qmicro, out=out, nt=nt_h, tf=tf_h)


def test_c2_every_query_every_method_vs_oracle(c2):
    from qppfuse import engine as e
    off_h = c2.off.cpu().numpy()
    doc_h = c2.docid.cpu().numpy().view(np.uint32)
    sc_h = c2.micro.cpu().numpy().astype(np.float64) / 1e6
    w_h = e.qpp_normalize(c2.qraw, c2.mm, c2.off, R, "minmax", 5,
                          want_micro=False)["weights"].cpu().numpy()
    out = c2.out
    uc = out.union_count.cpu().numpy()
    assert (uc > 3072).all() and uc.mean() > 3900, uc.mean()  # the large-union sort's range
    base = off_h[0:-1:R][:Q]
    idx = np.concatenate([np.arange(b, b + u) for b, u in zip(base, uc)])
    ud = out.union_docid.cpu().numpy().view(np.uint32)
    perm = out.perm.cpu().numpy().view(np.uint16)
    fz = out.fused.cpu().numpy()
    rk = out.ranked_fused().cpu().numpy()
    for m, name in enumerate(METHODS):
        o_ud, o_uc, o_perm, o_fused = coracle.fuse(off_h, doc_h, sc_h, R, name, 60,
                                                   weights=w_h if name.startswith("w") else None)
        assert np.array_equal(uc, o_uc), name
        if m == 0:
            assert np.array_equal(ud[idx], o_ud[idx])
        assert np.array_equal(perm[m, idx], o_perm[idx].astype(np.uint16)), name
        assert rk[m, idx].tobytes() == o_fused[idx].tobytes(), name  # ranked scores
        # first-seen order: fused[u] = the ranked score at the rank whose perm is u
        qpos = np.repeat(base, uc)
        first = np.zeros_like(fz[m])
        first[qpos + o_perm[idx].astype(np.int64)] = o_fused[idx]
        assert fz[m, idx].tobytes() == first[idx].tobytes(), name


def test_c2_qpp_file_values(c2):
    """All 13 normalised columns of every list, as the .qpp text holds them."""
    from qppfuse import engine as e
    dev = e.qpp_normalize(c2.qraw, c2.mm, c2.off, R, "minmax", 5)["micro"]
    assert torch.equal(c2.qmicro.view(-1), dev.reshape(-1))
    # the C restatement's raw predictors, normalised by numpy as src/qpp.py:356-361 and
    # formatted by Python's "%.6f" (src/qpp.py:333)
    off_h, raw_h = c2.off.cpu().numpy(), c2.raw.cpu().numpy()
    cut = [raw_h[off_h[l]:off_h[l + 1]][:100] for l in range(Q * R)]
    coff = np.cumsum([0] + [len(c) for c in cut]).astype(np.int64)
    want = coracle.qpp_raw(np.concatenate(cut), coff, np.repeat(c2.nt, R),
                           np.repeat(c2.tf[:, 0], R), np.repeat(c2.tf[:, 1], R))
    got = c2.qmicro.cpu().numpy().reshape(Q, R, 13)
    w = want.reshape(Q, R, 13)
    mismatch = 0
    for r in range(R):
        arr = w[:, r, :]
        mn, mx = arr.min(axis=0), arr.max(axis=0)
        scale = np.where(mx - mn > 0, mx - mn, 1.0)
        norm = (arr - mn) / scale
        text = np.array([[int(f"{x:.6f}".replace(".", "")) for x in row] for row in norm])
        mismatch += int((text != got[:, r, :]).sum())
    # the O(k) SigmaMax / CumNQC columns are within 1e-12 of Java's order
    # (tests/test_gpu_qpp_scale.py); on this batch no "%.6f" value moves
    assert mismatch == 0


def test_c2_large_query_path_identical(c2):
    """max_entries 7,680: the 768-thread join (JoinL, the path of queries of 5,121-7,680
    entries) with the same sorts gives the same outputs as the headline's JoinM."""
    from qppfuse import engine as e
    b = e.fuse(c2.off, c2.docid, c2.micro, R, METHODS, 60, max_entries=7680,
               qpp=(c2.qraw, c2.mm, "minmax", 5))
    a = c2.out
    off_h = c2.off.cpu().numpy()
    uc = a.union_count.cpu().numpy()
    idx = torch.from_numpy(np.concatenate([np.arange(s, s + u) for s, u in
                                           zip(off_h[0:-1:R][:Q], uc)])).to(a.fused.device)
    assert torch.equal(a.union_count, b.union_count)
    assert torch.equal(a.union_docid[idx], b.union_docid[idx])
    assert torch.equal(a.perm[:, idx], b.perm[:, idx])
    assert torch.equal(a.fused[:, idx].view(torch.int64), b.fused[:, idx].view(torch.int64))
