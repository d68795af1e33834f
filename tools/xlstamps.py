"""Phase breakdown of the workspace fusion kernel (join_sort_xl_kernel) from the
QF_STAMPS diagnostic build (development tool; build it first on the CPU with
`python tools/xlstamps.py --build`).  Cycles per query, summed over the blocks."""
import ctypes as C
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "qpp-fusion-rag_amd")]
LIB = ROOT / "qpp-fusion-rag_amd" / "qppfuse" / "libqppfuse_stamps.so"
if "--build" in sys.argv:
    from qppfuse import _build
    _build.build_variant(LIB, ["-DQF_STAMPS"])
    sys.exit(0)

import numpy as np
import torch

from qppfuse import _lib

_lib.LIB_PATH = LIB
from qppfuse import engine

lib = _lib.lib()
lib.qf_debug_stamps.restype = C.c_int
lib.qf_debug_stamps.argtypes = [C.c_void_p, C.c_int, C.c_int]
NB, NS = 32768, 16
names = ["init", "insert", "numbering", "group offsets", "placement", "sums",
         "sort:fill", "sort:tiles k<=T", "sort:global+tiles", "sort:output", "sort:bucket"]
args = [a for a in sys.argv[1:] if not a.startswith("-")]
Q, R, K = (int(a) for a in args) if len(args) == 3 else (3452, 16, 1000)
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
    # XL blocks 0..511; the LDS kernels return before their first stamp for
    # queries above their capacity, so these slots are the XL kernel's alone.
    st = buf.reshape(NB, NS)[:512, :11].astype(np.float64)
    out["+".join(ms)] = {n: round(float(st[:, i].sum() / Q)) for i, n in enumerate(names)}
print(json.dumps(out, indent=1))
