"""Per-kernel timing of the C2 pipeline (development tool, not the bench)."""
import sys, json
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "qpp-fusion-rag_amd")]
import os
import numpy as np, torch
from qppfuse import engine, _lib
if os.environ.get("QF_LIB"):  # A/B a development build of the same sources
    _lib.LIB_PATH = Path(os.environ["QF_LIB"])

def timeit(fn, n=10):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / n

Q, R, K = int(sys.argv[1]) if len(sys.argv) > 1 else 3452, 5, 1000
dev = torch.device("cuda", 0)
off, docid, raw = engine.synth_runs(0, Q, R, K)
norm, micro = engine.minmax_per_query(raw, off)
nt = torch.full((Q,), 4, dtype=torch.int32, device=dev)
tf = torch.rand((Q, 2), dtype=torch.float64, device=dev)
qraw = engine.qpp_raw(raw, off, R, 100, nt, tf)
mm = engine.qpp_colminmax(qraw, off, R)
w = engine.qpp_normalize(qraw, mm, off, R, "minmax", 5)["weights"]
res = {}
res["minmax"] = timeit(lambda: engine.minmax_per_query(raw, off, want_norm=False))
res["qpp_raw"] = timeit(lambda: engine.qpp_raw(raw, off, R, 100, nt, tf, out=qraw))
res["colminmax"] = timeit(lambda: engine.qpp_colminmax(qraw, off, R, out=mm))
res["normalize"] = timeit(lambda: engine.qpp_normalize(qraw, mm, off, R, "minmax", 5, want_micro=False))
for ms in (["rrf"], ["combsum"], ["wcombsum"], ["combsum", "rrf"], ["combsum", "combmnz", "rrf", "wcombsum", "wcombmnz", "wrrf"]):
    o = engine.alloc_fuse_out(Q, Q * R * K, engine.methods_mask(ms), dev)
    res["fuse:" + "+".join(ms)] = timeit(lambda: engine.fuse(off, docid, micro, R, ms, weights=w, max_entries=R * K, out=o))
uc = o.union_count.cpu().numpy()
res["mean_union"] = float(uc.mean()); res["min_uc"] = int(uc.min())
print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}))
