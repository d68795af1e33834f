"""Phase cycles of join_sort_kernel (QF_STAMPS build; development tool).

Per workgroup (= query), thread 0's s_memtime deltas, summed over the method
loop's iterations; slots: 3-7 join phases (join_groups), 0 the join in all,
8 sums + score ranges, 14 barrier into the sort (+ leftovers), 9 zeroing,
10 bucket parameters + barrier, 11 count, 12 barrier, 13 scan + barriers,
1 scatter + barrier, 2 rank + output, 15 loop-end barrier.
"""
import ctypes as C
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "qpp-fusion-rag_amd")]
import numpy as np
import torch
from qppfuse import _build, _lib

so = ROOT / "qpp-fusion-rag_amd" / "qppfuse" / "libqppfuse_stamps.so"
if not so.exists():
    raise SystemExit(f"build {so} first (qppfuse._build.build_variant, -DQF_STAMPS)")
_lib.LIB_PATH = so
from qppfuse import engine

lib = _lib.lib()
lib.qf_debug_stamps.restype = C.c_int
lib.qf_debug_stamps.argtypes = [C.c_void_p, C.c_int, C.c_int]
NB, NS = 32768, 16
names = {3: "join:load+init", 4: "join:insert", 5: "join:reps+scans", 6: "join:placement",
         7: "join:groups", 0: "join(all)", 8: "sums+ranges", 14: "bar+rest", 9: "zero",
         10: "params+bar", 11: "count", 12: "bar(count)", 13: "scan+bars", 1: "scatter+bar",
         2: "rank+out", 15: "bar(end)"}
Q, R, K = 3452, 5, 1000
dev = torch.device("cuda", 0)
off, docid, raw = engine.synth_runs(0, Q, R, K)
_, micro = engine.minmax_per_query(raw, off, want_norm=False)
w = torch.rand(Q * R, dtype=torch.float64, device=dev)
buf = np.zeros(NB * NS, np.uint64)
out = {}
for ms in (["rrf"], ["combsum", "combmnz", "rrf", "wcombsum", "wcombmnz", "wrrf"]):
    for rep in range(2):
        engine.fuse(off, docid, micro, R, ms, weights=w, max_entries=R * K)
        torch.cuda.synchronize()
        lib.qf_debug_stamps(buf.ctypes.data_as(C.c_void_p), NB * NS, 1)
    st = buf.reshape(NB, NS)[:Q].astype(np.float64)
    out["+".join(ms)] = {v: round(float(st[:, k].mean())) for k, v in names.items()}
    out["+".join(ms)]["total"] = round(float(st[:, [0, 8, 14, 9, 10, 11, 12, 13, 1, 2, 15]].sum(1).mean()))
Path("gpurun_out").mkdir(exist_ok=True)
Path("gpurun_out/js_stamps.json").write_text(json.dumps(out, indent=1))
print(json.dumps(out, indent=1))
