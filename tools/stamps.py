"""Phase breakdown of qf_fuse from the QF_STAMPS diagnostic build (development tool).

Reads per-block s_memtime deltas (shader cycles) of thread 0 at phase
boundaries; shares matter, not absolute length (stamps add fences).
"""
import ctypes as C
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "qpp-fusion-rag_amd")]
import numpy as np
import torch
from qppfuse import _lib

_lib.LIB_PATH = ROOT / "qpp-fusion-rag_amd" / "qppfuse" / "libqppfuse_stamps.so"
from qppfuse import engine

lib = _lib.lib()
lib.qf_debug_stamps.restype = C.c_int
lib.qf_debug_stamps.argtypes = [C.c_void_p, C.c_int, C.c_int]
NB, NS = 32768, 16
names = ["gather+keys", "sort", "output", "-", "-", "-", "-", "-", "cs:count", "cs:bar1", "cs:scan+bar", "cs:scatter", "cs:bar3", "cs:readback"]
Q, R, K = 3452, 5, 1000
dev = torch.device("cuda", 0)
off, docid, raw = engine.synth_runs(0, Q, R, K)
_, micro = engine.minmax_per_query(raw, off, want_norm=False)
w = torch.rand(Q * R, dtype=torch.float64, device=dev)
buf = np.zeros(NB * NS, np.uint64)
out = {}
for ms in (["rrf"], ["combsum", "combmnz", "rrf", "wcombsum", "wcombmnz", "wrrf"]):
    engine.fuse(off, docid, micro, R, ms, weights=w, max_entries=R * K)
    torch.cuda.synchronize()
    lib.qf_debug_stamps(buf.ctypes.data_as(C.c_void_p), NB * NS, 1)
    engine.fuse(off, docid, micro, R, ms, weights=w, max_entries=R * K)
    torch.cuda.synchronize()
    lib.qf_debug_stamps(buf.ctypes.data_as(C.c_void_p), NB * NS, 1)
    nb = ((Q + 7) // 8) * 8 * len(ms)
    st = buf.reshape(NB, NS)[:nb, :14].astype(np.float64)
    st = st[st[:, 0] > 0]  # blocks that ran (not padding / other pass)
    tot = st[:, :3].sum(1).mean()
    fx = buf.reshape(NB, NS)[Q:nb, 5:8].astype(np.float64)  # sort blocks only (join uses 3-7)
    fx = fx[fx[:, 1] > 0]
    fixup = {"fix:scan": round(float(fx[:, 0].mean())), "fix:barrier": round(float(fx[:, 1].mean())),
             "fix:runs+bar": round(float(fx[:, 2].mean())),
             "fix:blocks_with_runs": round(float((fx[:, 2] > 2000).mean()), 3)} if len(fx) else {}
    out["+".join(ms)] = {"cycles_per_block": round(tot), **fixup,
                         **{n: round(float(st[:, i].mean())) for i, n in enumerate(names)}}
    js = buf.reshape(NB, NS)[:Q].astype(np.float64)
    jn = {3: "join:load+init", 4: "join:insert", 5: "join:reps+scans", 6: "join:placement",
          7: "join:groups", 14: "join:sums+write"}
    # persistent join workgroups accumulate over their queries: per-query means
    out["join " + "+".join(ms)] = {v: round(float(js[:, k].sum() / Q)) for k, v in jn.items()}
Path("gpurun_out").mkdir(exist_ok=True)
Path("gpurun_out/stamps.json").write_text(json.dumps(out, indent=1))
print(json.dumps(out, indent=1))
