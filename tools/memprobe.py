"""Development probe: per-kernel times of the C3 path at a given query count
(python tools/memprobe.py Q [extra_GiB])."""
import sys, time
sys.path[:0] = ["/root/repo", "/root/repo/qpp-fusion-rag_amd"]
import torch
from qppfuse import engine

Q = int(sys.argv[1])
extra = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
pad = torch.empty(int(extra * 2**30), dtype=torch.uint8, device="cuda") if extra > 0 else None
R, K = 5, 1000


def timed(name, fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    print(f"Q={Q} {name}: {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
    return r


off, docid, raw = timed("synth", lambda: engine.synth_runs(0, Q, R, K))
for it in range(2):
    _, micro = timed("minmax", lambda: engine.minmax_per_query(raw, off, want_norm=False))
out = timed("fuse(alloc)", lambda: engine.fuse(off, docid, micro, R, ["combsum", "rrf"],
                                                 max_entries=R * K))
for it in range(2):
    timed("fuse", lambda: engine.fuse(off, docid, micro, R, ["combsum", "rrf"],
                                      max_entries=R * K, out=out))
