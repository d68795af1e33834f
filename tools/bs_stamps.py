"""Phase cycles of bucket_sort_kernel (QF_STAMPS build; development tool).

Slots per (query, method) workgroup (thread 0's s_memtime deltas): 0 load +
zero + barrier, 1 range + barrier, 2 count, 3 barrier, 4 scan + barriers,
5 scatter + barrier, 6 rank + output.  The join kernel's slots are not read.
"""
import ctypes as C
import json
import os
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
names = {0: "load+zero+bar", 1: "range+bar", 2: "count", 3: "bar(count)", 4: "scan+bars",
         5: "scatter+bar", 6: "rank+out"}
Q, R, K = 3452, 5, 1000
dev = torch.device("cuda", 0)
off, docid, raw = engine.synth_runs(0, Q, R, K)
_, micro = engine.minmax_per_query(raw, off, want_norm=False)
w = torch.rand(Q * R, dtype=torch.float64, device=dev)
buf = np.zeros(NB * NS, np.uint64)
M = ["combsum", "combmnz", "rrf", "wcombsum", "wcombmnz", "wrrf"]
for rep in range(2):
    engine.fuse(off, docid, micro, R, M, weights=w, max_entries=R * K)
    torch.cuda.synchronize()
    lib.qf_debug_stamps(buf.ctypes.data_as(C.c_void_p), NB * NS, 1)
nb = min(NB, ((Q + 7) // 8) * 8 * len(M))
st = buf.reshape(NB, NS)[:nb].astype(np.float64)
st = st[st[:, 6] > 0]
out = {v: round(float(st[:, k].mean())) for k, v in names.items()}
out["total"] = round(float(st[:, list(names)].sum(1).mean()))
out["blocks"] = int(len(st))
Path("gpurun_out").mkdir(exist_ok=True)
Path("gpurun_out/bs_stamps.json").write_text(json.dumps(out, indent=1))
print(json.dumps(out, indent=1))
