"""The LDS join's hash insert under worst-case collisions — needs an MI355X.

Every docid of a query is chosen to land on the same home slot of the join's table
(slot = top TB bits of docid * 0x9E3779B1, csrc/qf_fuse.hip join_groups), so each
insert walks the triangular probe sequence past every key placed before it: the
longest chains the join can see, on each LDS configuration (one-wave JoinT, JoinS,
JoinM, JoinL).  The fused lists must still equal the C oracle's bit for bit.
"""
import numpy as np
import pytest
import torch

from oracle import _loader as coracle

pytestmark = pytest.mark.gpu

ALL = ["combsum", "combmnz", "rrf", "wcombsum", "wcombmnz", "wrrf"]
_INV_PHI = pow(0x9E3779B1, -1, 1 << 32)  # docid * 0x9E3779B1 = (slot << (32 - TB)) | j


def _colliding_ids(tb: int, slot: int, n: int) -> np.ndarray:
    j = np.arange(n, dtype=np.uint64)
    d = ((np.uint64(slot) << np.uint64(32 - tb)) | j) * np.uint64(_INV_PHI) & np.uint64(0xFFFFFFFF)
    d = d.astype(np.uint32)
    assert ((d.astype(np.uint64) * 0x9E3779B1 & 0xFFFFFFFF) >> (32 - tb) == slot).all()
    return d[d != 0xFFFFFFFF]


def _runs(Q, R, K, tb, seed):
    """R lists of K distinct colliding docids per query (lists overlap: a pool of
    ~0.8 R K ids), micro-unit scores strictly decreasing in each list."""
    rng = np.random.default_rng(seed)
    off = np.zeros(Q * R + 1, np.int64)
    docs, micro = [], []
    for q in range(Q):
        pool = _colliding_ids(tb, int(rng.integers(0, 1 << tb)), max(K, int(0.8 * R * K)))
        for r in range(R):
            docs.append(rng.choice(pool, K, replace=False))
            s = np.sort(rng.choice(1_000_001, K, replace=False))[::-1]
            micro.append(s.astype(np.int32))
            off[q * R + r + 1] = off[q * R + r] + K
    return off, np.concatenate(docs), np.concatenate(micro)


@pytest.mark.parametrize("shape", [(32, 3, 100, 10),   # N 300: JoinT (one wave, 2^10 slots)
                                   (16, 4, 250, 11),   # N 1,000: JoinS (2^11)
                                   (16, 5, 1000, 13),  # N 5,000: JoinM (2^13), C2's shape
                                   (6, 7, 1000, 14)])  # N 7,000: JoinL (2^14)
def test_join_all_keys_on_one_home_slot(gpu, shape):
    from qppfuse import engine
    Q, R, K, tb = shape
    off_h, doc_h, mic_h = _runs(Q, R, K, tb, seed=Q * R + K)
    off = torch.from_numpy(off_h).to(gpu)
    docid = torch.from_numpy(doc_h.view(np.int32)).to(gpu)
    micro = torch.from_numpy(mic_h).to(gpu)
    w_h = np.random.default_rng(K).random(Q * R).round(6)
    w = torch.from_numpy(w_h).to(gpu)
    out = engine.fuse(off, docid, micro, R, ALL, rrf_k=60, weights=w, max_entries=R * K)
    torch.cuda.synchronize()
    sc_h = mic_h.astype(np.float64) / 1e6
    ud = out.union_docid.cpu().numpy().view(np.uint32)
    uc = out.union_count.cpu().numpy()
    perm = out.perm.cpu().numpy().view(np.uint32 if out.wide else np.uint16)
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
