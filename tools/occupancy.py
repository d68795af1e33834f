"""qf_fuse time vs workgroups per CU (QF_LDS_PAD forces 1/CU) and vs batch size."""
import os, sys, json, subprocess
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
code = r'''
import sys, json
sys.path[:0] = ["%s", "%s/qpp-fusion-rag_amd"]
import torch
from qppfuse import engine
def t(fn, n=10):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n): fn()
    b.record(); torch.cuda.synchronize(); return a.elapsed_time(b) / n
R, K = 5, 1000
res = {}
for Q in (256, 512, 1024, 3452, 6904):
    off, docid, raw = engine.synth_runs(0, Q, R, K)
    _, micro = engine.minmax_per_query(raw, off, want_norm=False)
    w = torch.rand(Q * R, dtype=torch.float64, device="cuda")
    ms = ["combsum", "combmnz", "rrf", "wcombsum", "wcombmnz", "wrrf"]
    o = engine.alloc_fuse_out(Q, Q * R * K, engine.methods_mask(ms), "cuda")
    res[Q] = round(t(lambda: engine.fuse(off, docid, micro, R, ms, weights=w, max_entries=R * K, out=o)), 4)
print(json.dumps(res))
''' % (ROOT, ROOT)
for pad in ("0", "70000"):
    env = dict(os.environ, QF_LDS_PAD=pad)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True)
    print("pad", pad, r.stdout.strip(), r.stderr.strip()[-300:] if r.returncode else "")
