"""Does pipelining consecutive C2 batches pay?  Step i's fusion (qf_fuse) on the main
stream beside step i+1's QPP + min-max + normalisation on a side stream (two
buffer sets, event-ordered), against the serial step.  Development probe: prints
ms per step both ways and whether the last step's outputs are identical."""
import hashlib
import json
import sys
import time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "qpp-fusion-rag_amd")]
import torch
from qppfuse import engine, _lib

dev = torch.device("cuda", 0)
Q, R, K = 3452, 5, 1000
M = ["combsum", "combmnz", "rrf", "wcombsum", "wcombmnz", "wrrf"]
off, docid, raw = engine.synth_runs(0, Q, R, K)
nt = torch.full((Q,), 4, dtype=torch.int32, device=dev)
tf = torch.rand((Q, 2), dtype=torch.float64, device=dev)
E = Q * R * K
bufs = [dict(micro=torch.empty(E, dtype=torch.int32, device=dev),
             qraw=torch.empty((Q * R, 13), dtype=torch.float64, device=dev),
             mm=torch.empty(2 * R * 13, dtype=torch.float64, device=dev),
             w=None) for _ in range(2)]
out = engine.alloc_fuse_out(Q, E, engine.methods_mask(M), dev)


def prep(b):
    s = torch.cuda.current_stream().cuda_stream
    engine.qpp_raw(raw, off, R, 100, nt, tf, out=b["qraw"])
    engine.qpp_colminmax(b["qraw"], off, R, out=b["mm"])
    _lib.call("qf_minmax_per_query", raw.data_ptr(), off.data_ptr(), Q * R, None,
              b["micro"].data_ptr(), s)
    b["w"] = engine.qpp_normalize(b["qraw"], b["mm"], off, R, "minmax", 5, want_micro=False)["weights"]


def fuse(b):
    engine.fuse(off, docid, b["micro"], R, M, 60, weights=b["w"], max_entries=R * K, out=out)


def digest():
    h = hashlib.sha256(out.union_count.cpu().numpy().tobytes())
    h.update(out.fused.cpu().numpy().tobytes())
    h.update(out.perm.cpu().numpy().tobytes())
    return h.hexdigest()[:16]


def serial(n):
    for _ in range(n):
        prep(bufs[0])
        fuse(bufs[0])


side = torch.cuda.Stream(device=dev)
main = torch.cuda.current_stream()


def overlapped(n):
    ready = [torch.cuda.Event(), torch.cuda.Event()]
    freed = [torch.cuda.Event(), torch.cuda.Event()]
    with torch.cuda.stream(side):
        prep(bufs[0])
        ready[0].record(side)
    for i in range(n):
        cur, nxt = i % 2, (i + 1) % 2
        if i + 1 < n:
            with torch.cuda.stream(side):
                if i >= 1:
                    side.wait_event(freed[nxt])  # fuse(i - 1) done with this set
                prep(bufs[nxt])
                ready[nxt].record(side)
        main.wait_event(ready[cur])
        fuse(bufs[cur])
        freed[cur].record(main)


res = {}
for name, fn in (("serial", serial), ("overlapped", overlapped), ("serial2", serial),
                 ("overlapped2", overlapped)):
    fn(20)
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn(200)
    torch.cuda.synchronize()
    res[name + "_ms"] = round((time.perf_counter() - t) / 200 * 1e3, 4)
    res[name + "_digest"] = digest()
print(json.dumps(res))
