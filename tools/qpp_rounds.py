"""qf_qpp_raw time against the number of lists: 8 lists per 512-thread workgroup, 4
workgroups per CU -> 8,192 lists fill the GPU once.  Does the partial last round of
C2's 17,260 lists (2.1 fills) cost a whole round?  (development probe)"""
import json
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "qpp-fusion-rag_amd")]
import torch
from qppfuse import engine

dev = torch.device("cuda", 0)
R, K = 5, 1000
res = {}
for Q in (819, 1638, 2457, 3276, 3452, 4096, 4915, 6553):
    off, docid, raw = engine.synth_runs(0, Q, R, K)
    nt = torch.full((Q,), 4, dtype=torch.int32, device=dev)
    tf = torch.rand((Q, 2), dtype=torch.float64, device=dev)
    out = engine.qpp_raw(raw, off, R, 100, nt, tf)
    for _ in range(3):
        engine.qpp_raw(raw, off, R, 100, nt, tf, out=out)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        engine.qpp_raw(raw, off, R, 100, nt, tf, out=out)
    b.record()
    torch.cuda.synchronize()
    res[Q * R] = round(a.elapsed_time(b) / 20 * 1e3, 1)
    del off, docid, raw
print(json.dumps({"lists_to_us": res, "fills_of_8192_lists": {k: round(k / 8192, 2) for k in res}}))
