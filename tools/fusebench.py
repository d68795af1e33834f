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
if os.environ.get("FUSEBENCH_SYNTH", "nq") == "nq":  # SURVEY §8(d)'s generator (bench default)
    sys.path.insert(0, str(ROOT))
    import bench
    qo, qd = bench.nq_qrels()
    off, docid, raw = engine.synth_runs_nq(0, Q, R, K, qo, qd)
else:  # rounds 1-4's generator
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
# (raw buffers, no gather through perm: a development build that stops before the
# sort's stores leaves perm uninitialised, and an index through it could fault)
# (gathered on the host, over the slots each query owns: a development build that
# stops before the sort's stores leaves perm uninitialised, and a device gather
# through it could fault)
uc = out.union_count.cpu().numpy()
h = hashlib.sha256(uc.tobytes())
perm, fused, lo = out.perm.cpu().numpy(), out.fused.cpu().numpy(), off.cpu().numpy()
for q in range(Q):
    b, u = int(lo[q * R]), int(uc[q])
    if u > 0:
        h.update(perm[:, b:b + u].tobytes())
        h.update(fused[:, b:b + u].tobytes())
print("ok", h.hexdigest()[:16])
