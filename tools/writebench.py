"""write_run (the native writer) on a C2-sized fused run: 3,452 queries x 2,500
documents, 390 MB of text (development tool; QFIO_WRITE_PWRITE=1 for the pwrite A/B)."""
import os
import sys
import tempfile
import time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "qpp-fusion-rag_amd")]
import numpy as np
from qppfuse import fastio
from qppfuse.runset import RunSet
rng = np.random.default_rng(0)
Q, U = 3452, 2500
E = Q * 5000
qids = [f"test{i}" for i in range(Q)]
docnos = np.array([f"doc{i:08d}" for i in range(Q * U)], dtype=object)
qbase = np.arange(Q, dtype=np.int64) * 5000
counts = np.full(Q, U, np.int32)
ud = np.zeros(E, np.uint32); perm = np.zeros(E, np.uint16); fused = np.zeros(E)
for q in range(Q):
    b = q * 5000
    ud[b:b+U] = np.arange(q * U, (q + 1) * U)
    perm[b:b+U] = rng.permutation(U)
    fused[b:b+U] = rng.random(U) * 3
rs = RunSet(qids=qids, rankers=["a"], docnos=docnos, list_off=np.zeros(2, np.int64),
            docid=np.zeros(0, np.uint32), score=np.zeros(0), rank=np.zeros(0, np.int64))
order = np.arange(Q, dtype=np.int64)
OUT = os.path.join(tempfile.gettempdir(), "qf_writebench.res")
fastio.write_run(OUT, order, qbase, counts, ud, perm, fused, rs, "combsum")
ts = []
for i in range(5):
    t = time.perf_counter()
    fastio.write_run(OUT, order, qbase, counts, ud, perm, fused, rs, "combsum")
    ts.append(time.perf_counter() - t)
print("write_run s", [round(x, 3) for x in ts], os.path.getsize(OUT) / 1e6, "MB")
