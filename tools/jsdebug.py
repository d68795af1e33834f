"""Development: compare qf_fuse's fused join+sort path with the C oracle, query by query."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "qpp-fusion-rag_amd")]
import numpy as np
import torch
from qppfuse import engine
from oracle import _loader as coracle

Q, R, K = int(sys.argv[1]) if len(sys.argv) > 1 else 16, 5, 400
off, docid, raw = engine.synth_runs(0, Q, R, K, seed=11, p_shared=0.7)
_, micro = engine.minmax_per_query(raw, off, want_norm=False)
methods = ["combsum", "combmnz", "rrf", "wcombsum", "wcombmnz", "wrrf"]
torch.manual_seed(0)
w = torch.rand(Q * R, dtype=torch.float64, device="cuda")
out = engine.fuse(off, docid, micro, R, methods, weights=w, max_entries=R * K)
torch.cuda.synchronize()
off_h = off.cpu().numpy(); doc_h = docid.cpu().numpy().view(np.uint32)
sc = micro.cpu().numpy().astype(np.float64) / 1e6
uc = out.union_count.cpu().numpy()
perm = out.perm.cpu().numpy().view(np.uint16); fz = out.ranked_fused().cpu().numpy()
bad = 0
for m, name in enumerate(methods):
    _, o_uc, o_perm, o_fused = coracle.fuse(off_h, doc_h, sc, R, name, 60, weights=w.cpu().numpy())
    for q in range(Q):
        b, n = off_h[q * R], uc[q]
        if n != o_uc[q]:
            print(name, q, "U", n, o_uc[q]); bad += 1; continue
        gp, op = perm[m, b:b + n], o_perm[b:b + n]
        gv, ov = fz[m, b:b + n], o_fused[b:b + n]
        if not (np.array_equal(gp, op) and gv.tobytes() == ov.tobytes()):
            bad += 1
            d = np.nonzero((gp != op) | (gv != ov))[0]
            print(f"{name} q{q} U={n}: {len(d)} diffs, first at {d[:8]}")
            for i in d[:4]:
                print(f"   pos {i}: got u={gp[i]} v={gv[i]!r}  want u={op[i]} v={ov[i]!r}")
            print("   got perm unique:", len(set(gp.tolist())), "marker count", int((gp == 0xFFFF).sum()))
print("bad", bad)
