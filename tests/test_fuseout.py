"""FuseOut.ranked_fused (CPU tensors): qf_fuse keeps the scores in first-seen order
and ranks them with perm; the rank-order view gathers fused[b + perm[b + i]] per
query and zero-fills the slots past each union."""
import numpy as np
import torch

from qppfuse.engine import FuseOut


def test_ranked_fused_gathers_through_perm():
    rng = np.random.default_rng(3)
    R, sizes = 2, [5, 0, 7, 3]           # entries per query (two lists each)
    lens = [[s // 2, s - s // 2] for s in sizes]
    off = np.concatenate([[0], np.cumsum(np.ravel(lens))]).astype(np.int64)
    E, M = int(off[-1]), 2
    U = np.array([4, 0, 7, 1], np.int32)  # unions (<= entries)
    fused = rng.standard_normal((M, E))
    perm = np.zeros((M, E), np.int16)
    want = np.zeros((M, E))
    for q in range(len(sizes)):
        b = off[q * R]
        for m in range(M):
            p = rng.permutation(U[q])
            perm[m, b:b + U[q]] = p
            want[m, b:b + U[q]] = fused[m, b + p]
    out = FuseOut(torch.zeros(E, dtype=torch.int32), torch.from_numpy(U),
                  torch.from_numpy(perm), torch.from_numpy(fused), ["a", "b"],
                  torch.from_numpy(off), R)
    got = out.ranked_fused().numpy()
    assert got.tobytes() == want.tobytes()
