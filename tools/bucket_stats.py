"""Bucket-size statistics of the bucket sort's key on dumped C2 fusions (development).

Input: gpurun_out/fused_c2.npz from tools/dump_fused.py (200 queries' inputs and
QPP weights).  Fuses them with the C oracle (QPP weights and uniform random
weights) and reports, for several delta = range / 2^k: mean in-bucket loop per
item, mean per-wave largest bucket, largest bucket, queries over kJsBucketMax.
"""
import sys; from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / 'qpp-fusion-rag_amd')]
import numpy as np
from oracle import _loader as coracle
d = np.load(ROOT / "gpurun_out" / "fused_c2.npz")
off, micro, docid = d["off"], d["micro"], d["docid"].view(np.uint32)
R = 5; Q = 200
off = off[:Q*R+1]; n = off[-1]
sc = micro[:n].astype(np.float64)/1e6
NB, MINSUB = 4096, 256; MINBASE = NB - MINSUB
def stats(fz, uc, k):
    mx_all = []; loops = []; wmax = []; over = 0
    for q in range(Q):
        b, U = off[q*R], uc[q]
        v = fz[b:b+U]
        lo, hi = v.min(), v.max(); rngv = hi - lo; delta = rngv * 2.0**-k
        b0 = np.float32(delta).view(np.uint32).astype(np.int64)
        span = np.float32(rngv + delta).view(np.uint32).astype(np.int64) - b0
        bsh = max(0, int(span).bit_length() - 12)
        if (span >> bsh) >= MINBASE: bsh += 1
        x = ((v - lo) + delta).astype(np.float32).view(np.uint32).astype(np.int64)
        u = np.arange(U)
        wv = np.where(v == lo, MINBASE + np.minimum((u * np.float32(MINSUB / U)).astype(np.int64), MINSUB-1), MINBASE - 1 - ((x - b0) >> bsh))
        c = np.bincount(wv, minlength=NB); mx_all.append(c.max()); over += c.max() > 128
        loops.append((c.astype(float)**2).sum()/U)
        cs = np.sort(wv); cc = c[cs]; pad = (-len(cc)) % 64
        wmax.append(np.pad(cc,(0,pad)).reshape(-1,64).max(1).mean())
    return np.mean(loops), np.mean(wmax), np.max(mx_all), over
rng = np.random.default_rng(0)
for wname, w in [("qpp", d["w"][:Q*R]), ("rand", rng.random(Q*R))]:
    for name in ["combsum","combmnz","rrf","wcombsum","wcombmnz","wrrf"]:
        if wname == "rand" and not name.startswith("w"): continue
        ud, uc, perm, fz = coracle.fuse(off, docid[:n], sc, R, name, 60, weights=w)
        row = []
        for k in (5, 8, 12, 16, 24):
            L, W, M, O = stats(fz, uc, k)
            row.append(f"k{k}: {L:.2f}/{W:.1f}/max{M}/o{O}")
        print(f"{wname} {name:9s} " + "  ".join(row))
