"""C2-scale QPP parity — needs an MI355X.

qpp_raw_kernel takes SigmaMax (col 3) and CumNQC (col 9) from O(k) Welford prefix
statistics instead of Java's O(k^2) from-scratch prefixes (QPPBridge.java:269-293,
400-410; csrc/qf_qpp.hip).  On the bench's C2 workload (3,452 queries x 5 retrievers
x 1,000, both synthetic generators, k = min(50, top-100)) against the exact Java
restatement (oracle/qpp_oracle.c):
  * every raw column within 1e-12 relative (RTOL below; ATOL only for values that
    are themselves ~0);
  * every "%.6f" .qpp value identical: the device normalisation of the device raw
    predictors == that of the oracle's raw predictors, micro-unit for micro-unit;
  * every W-* fusion bit-identical: wcombsum / wcombmnz / wrrf with the RSD weights
    (qpp_index 5, the default) and the 13-column mean (-1) from either raw set.
"""
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from oracle import _loader as coracle

pytestmark = pytest.mark.gpu

RTOL, ATOL = 1e-12, 1e-15
Q, R, K = 3452, 5, 1000


def _valid_slots(off: np.ndarray, ucount: np.ndarray) -> np.ndarray:
    """The entry positions b + u (u < union_count) of every query: the slots qf_fuse
    defines (the rest of each query's range is scratch)."""
    b = off[0:-1:R]
    return np.concatenate([np.arange(s, s + u) for s, u in zip(b, ucount)])


@pytest.mark.parametrize("generator", ["nq", "legacy"])
def test_qpp_c2_scale(gpu, generator):
    import bench
    from qppfuse import engine as e
    off, docid, raw = bench.gen_runs(SimpleNamespace(generator=generator), 0, Q, R, K)
    nt_h, tf_h = bench.text_inputs(0, Q)
    nt, tf = torch.from_numpy(nt_h).to(gpu), torch.from_numpy(tf_h).to(gpu)
    qraw = e.qpp_raw(raw, off, R, 100, nt, tf)

    off_h, raw_h = off.cpu().numpy(), raw.cpu().numpy()
    cut = [raw_h[off_h[l]:off_h[l + 1]][:100] for l in range(Q * R)]
    coff = np.cumsum([0] + [len(c) for c in cut]).astype(np.int64)
    want = coracle.qpp_raw(np.concatenate(cut), coff, np.repeat(nt_h, R),
                           np.repeat(tf_h[:, 0], R), np.repeat(tf_h[:, 1], R))
    got = qraw.cpu().numpy()
    np.testing.assert_allclose(got, want, rtol=RTOL, atol=ATOL)
    # Java's order and no libm call: NQC, WIG, SigmaX, UEF and the text columns are
    # bit-identical (SMV / RSD / SNQC / dense-qpp differ by libm ulps at most, and
    # SigmaMax / CumNQC are the O(k) ones)
    bit = [0, 2, 4, 6, 7, 8]
    assert got[:, bit].tobytes() == want[:, bit].tobytes()

    qw = torch.from_numpy(want).to(gpu)
    mm_g, mm_w = e.qpp_colminmax(qraw, off, R), e.qpp_colminmax(qw, off, R)
    _, micro = e.minmax_per_query(raw, off, want_norm=False)
    methods = ["wcombsum", "wcombmnz", "wrrf"]
    for idx in (5, -1):
        a = e.qpp_normalize(qraw, mm_g, off, R, "minmax", idx)
        b = e.qpp_normalize(qw, mm_w, off, R, "minmax", idx)
        assert torch.equal(a["micro"], b["micro"]), idx  # every "%.6f" .qpp value
        assert torch.equal(a["weights"].view(torch.int64), b["weights"].view(torch.int64))
        fa = e.fuse(off, docid, micro, R, methods, 60, weights=a["weights"], max_entries=R * K)
        fb = e.fuse(off, docid, micro, R, methods, 60, weights=b["weights"], max_entries=R * K)
        assert torch.equal(fa.union_count, fb.union_count)
        idx_t = torch.from_numpy(_valid_slots(off_h, fa.union_count.cpu().numpy())).to(gpu)
        assert torch.equal(fa.fused[:, idx_t].view(torch.int64), fb.fused[:, idx_t].view(torch.int64))
        assert torch.equal(fa.perm[:, idx_t], fb.perm[:, idx_t])
