"""Digest of qf_qpp_raw's output on C2's synthetic run set (and a ragged set with
short lists), plus its kernel time: equal digests across two builds (QPPFUSE_LIB)
mean bit-identical predictors.  Development A/B tool."""
import hashlib
import json
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "qpp-fusion-rag_amd")]
import numpy as np
import torch
from qppfuse import engine

dev = torch.device("cuda", 0)
Q, R, K = 3452, 5, 1000
off, docid, raw = engine.synth_runs(0, Q, R, K)
nt = torch.full((Q,), 4, dtype=torch.int32, device=dev)
tf = torch.rand((Q, 2), dtype=torch.float64, device=dev, generator=torch.Generator(dev).manual_seed(3))
h = hashlib.sha256()
out = engine.qpp_raw(raw, off, R, 100, nt, tf)
h.update(out.cpu().numpy().tobytes())
# ragged lists (1..120 entries, some empty) with ties
rng = np.random.default_rng(5)
lens = rng.integers(0, 120, 4000)
lens[::37] = 0
vals = np.concatenate([np.sort(np.round(rng.gamma(2, 3, n), 2))[::-1] for n in lens])
o2 = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)).to(dev)
q2 = len(lens) // 4
out2 = engine.qpp_raw(torch.from_numpy(vals).to(dev), o2, 4, 100,
                      nt[:q2].contiguous() if q2 <= Q else torch.full((q2,), 4, dtype=torch.int32, device=dev),
                      tf[:q2].contiguous())
h.update(out2.cpu().numpy().tobytes())
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(5):
    engine.qpp_raw(raw, off, R, 100, nt, tf, out=out)
a.record()
for _ in range(50):
    engine.qpp_raw(raw, off, R, 100, nt, tf, out=out)
b.record()
torch.cuda.synchronize()
print(json.dumps({"digest": h.hexdigest()[:16], "qpp_raw_ms": round(a.elapsed_time(b) / 50, 4)}))
