"""Phase cycles of bucket_sort_kernel (QF_STAMPS build; development tool).

Slots per (query, method) workgroup (thread 0's s_memtime deltas): 8 load +
zero, 9 range + barrier, 10 count, 11 barrier, 12 scan + barriers, 13 scatter +
barrier, 2 rank, 15 output; the join kernel's (per query): 3-7 join_groups'
phases, 14 sums + unsorted writes.
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
names = {8: "load+zero", 9: "range+bar", 10: "count", 11: "bar(count)", 12: "scan+bars",
         13: "scatter+bar", 2: "rank", 15: "out"}
jnames = {3: "join:load+init", 4: "join:insert", 5: "join:reps+scans", 6: "join:placement",
          7: "join:groups", 14: "join:sums+write"}
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
st = st[st[:, 15] > 0]
out = {v: round(float(st[:, k].mean())) for k, v in names.items()}
js = buf.reshape(NB, NS)[:Q].astype(np.float64)
out.update({v: round(float(js[:, k].mean())) for k, v in jnames.items()})
out["join_total"] = round(float(js[:, list(jnames)].sum(1).mean()))
out["total"] = round(float(st[:, list(names)].sum(1).mean()))
out["blocks"] = int(len(st))
Path("gpurun_out").mkdir(exist_ok=True)
Path("gpurun_out/bs_stamps.json").write_text(json.dumps(out, indent=1))
print(json.dumps(out, indent=1))
