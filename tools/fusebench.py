"""Only the C2 six-method qf_fuse launch, repeated (development: PMC passes)."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "qpp-fusion-rag_amd")]
import os
if os.environ.get("QF_LIB"):  # a development build of the same sources
    os.environ["QPPFUSE_LIB"] = os.environ["QF_LIB"]
import torch
from qppfuse import engine, _lib
Q, R, K = 3452, 5, 1000
dev = torch.device("cuda", 0)
off, docid, raw = engine.synth_runs(0, Q, R, K)
_, micro = engine.minmax_per_query(raw, off, want_norm=False)
torch.manual_seed(7)
w = torch.rand(Q * R, dtype=torch.float64, device=dev)
M = os.environ.get("FUSEBENCH_METHODS", "combsum,combmnz,rrf,wcombsum,wcombmnz,wrrf").split(",")
out = engine.alloc_fuse_out(Q, Q * R * K, engine.methods_mask(M), dev)
for _ in range(5):
    engine.fuse(off, docid, micro, R, M, weights=w, max_entries=R * K, out=out)
torch.cuda.synchronize()
# a digest of the outputs (union sizes + every ranked list): equal across libraries
# means the same results
import hashlib
h = hashlib.sha256(out.union_count.cpu().numpy().tobytes())
h.update(out.ranked_fused().cpu().numpy().tobytes())
print("ok", h.hexdigest()[:16])
