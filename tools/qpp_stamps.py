"""Phase cycles of qf_qpp_raw from the QF_STAMPS diagnostic build (development tool).

Per workgroup, wave 0's s_memtime deltas between the kernel's barriers: 1 = loads +
rsv to LDS, 2 = serial prefix chains (waves 0-1), 3 = per-prefix deviations + per-element
terms, 4 = the batched left-to-right sums.  Shares matter, not absolute length.
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
lib.qf_debug_qpp_stamps.restype = C.c_int
lib.qf_debug_qpp_stamps.argtypes = [C.c_void_p, C.c_int, C.c_int]
NB, NS = 4096, 8
Q, R, K = 3452, 5, 1000
dev = torch.device("cuda", 0)
off, docid, raw = engine.synth_runs(0, Q, R, K)
nt = torch.full((Q,), 4, dtype=torch.int32, device=dev)
tf = torch.rand((Q, 2), dtype=torch.float64, device=dev)
buf = np.zeros(NB * NS, np.uint64)
engine.qpp_raw(raw, off, R, 100, nt, tf)
torch.cuda.synchronize()
lib.qf_debug_qpp_stamps(buf.ctypes.data_as(C.c_void_p), NB * NS, 1)
engine.qpp_raw(raw, off, R, 100, nt, tf)
torch.cuda.synchronize()
lib.qf_debug_qpp_stamps(buf.ctypes.data_as(C.c_void_p), NB * NS, 1)
nwg = (Q * R + 7) // 8
st = buf.reshape(NB, NS)[:nwg, 1:5].astype(np.float64)
tot = st.sum(1)
out = {"workgroups": nwg, "cycles_per_wg_mean": round(float(tot.mean())),
       "cycles_per_wg_p10_p50_p90": [round(float(np.percentile(tot, x))) for x in (10, 50, 90)],
       **{n: round(float(st[:, i].mean())) for i, n in
          enumerate(["1:loads", "2:serial_prefix", "3:deviations+terms", "4:serial_sums"])}}
print(json.dumps(out))
