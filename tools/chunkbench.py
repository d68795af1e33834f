"""qf_fuse over the C2 batch in query chunks (development: does a chunk's
join -> sort intermediate staying in the MALL pay for the extra launches?)."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "qpp-fusion-rag_amd")]
import json
import numpy as np
import torch
from qppfuse import engine, _lib

Q, R, K = 3452, 5, 1000
dev = torch.device("cuda", 0)
off, docid, raw = engine.synth_runs(0, Q, R, K)
_, micro = engine.minmax_per_query(raw, off, want_norm=False)
w = torch.rand(Q * R, dtype=torch.float64, device=dev)
M = ["combsum", "combmnz", "rrf", "wcombsum", "wcombmnz", "wrrf"]
mask = engine.methods_mask(M)
out = engine.alloc_fuse_out(Q, Q * R * K, mask, dev)
st = lambda: torch.cuda.current_stream().cuda_stream


def run(chunks):
    b = np.linspace(0, Q, chunks + 1).astype(int)
    for c in range(chunks):
        q0, q1 = int(b[c]), int(b[c + 1])
        _lib.call("qf_fuse", q1 - q0, R, off.data_ptr() + 8 * q0 * R, docid.data_ptr(),
                  micro.data_ptr(), _lib.SCORE_MICRO, None, w.data_ptr() + 8 * q0 * R, mask, 60,
                  R * K, out.union_docid.data_ptr(), out.union_count.data_ptr() + 4 * q0,
                  out.perm.data_ptr(), out.fused.data_ptr(), out.fused.shape[1], st())


res = {}
for chunks in (1, 2, 3, 4, 8):
    run(chunks)
    torch.cuda.synchronize()
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        run(chunks)
    e.record()
    torch.cuda.synchronize()
    res[chunks] = round(a.elapsed_time(e) / 10, 4)
print(json.dumps(res))
