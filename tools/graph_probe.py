"""Eager vs hipGraph-replayed bench step (development probe): python tools/graph_probe.py c1|c2"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "qpp-fusion-rag_amd")]
import torch  # noqa: E402
import bench  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
sys.argv = ["bench.py", "--workload", wl]
args = bench.parse()
args.gather_topk = 0
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
from qppfuse import _lib  # noqa: E402
_lib.lib()
p = bench.Pipeline(args, 1, 0, dev)
for _ in range(3):
    p.step()
torch.cuda.synchronize()
K = 200


def timed(fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(K):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / K * 1e3


eager = timed(lambda: p.step())
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    p.step()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
with torch.cuda.graph(g):
    p.step()
torch.cuda.synchronize()
graph = timed(lambda: g.replay())
eager2 = timed(lambda: p.step())
ok = bench.check_parity(p, 8)
K = 20
eager20 = timed(lambda: p.step())
ev20 = timed(lambda: p.step(timed=True))
K = 200
ev200 = timed(lambda: p.step(timed=True))
loop20 = bench.timed_loop(p, 20, 1, dev) / 20 * 1e3
print({"workload": wl, "eager_ms": round(eager, 4), "graph_ms": round(graph, 4),
       "eager2_ms": round(eager2, 4), "parity_after_graph": ok, "eager_k20": round(eager20, 4),
       "events_k20": round(ev20, 4), "events_k200": round(ev200, 4),
       "bench_timed_loop_k20": round(loop20, 4)})
