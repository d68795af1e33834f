"""Offline model of bsort_kernel's rank-loop cost on C2-shaped synthetic data
(development): the numpy synthetic runs (tools/synth_np.py), the C oracle's fused
scores, bsort's bucket function, and per (wave, row) the largest bucket — the rank
loop's trip count.  Prints per method: mean U, mean buckets, mean largest bucket per
(wave, row), modelled rank-loop VALU per wave.  Usage: python tools/bsort_sim.py [Q]"""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tools")]
import numpy as np
from oracle import _loader as co
from synth_np import synth

Q = int(sys.argv[1]) if len(sys.argv) > 1 else 100
R, K, NB, BLOCK = 5, 1000, 4096, 512
MINSUB = NB // 16
MINBASE = NB - MINSUB
off, docid, raw = synth(0, Q, R, K)
norm = co.minmax_per_query(raw, off)
sc = np.round(norm * 1e6) / 1e6
rng = np.random.default_rng(7)
w = rng.random(Q * R)


def hi32(x):
    return (np.asarray(x, np.float64).view(np.uint64) >> np.uint64(32)).astype(np.int64)


def buckets(v, shift=8):
    """bsort_kernel's bucket of every item (csrc/qf_fuse.hip): x = v + c (or the
    difference form), the high word of x's bits, scaled onto MINBASE buckets by a
    multiply-high; the minimum's items by u >> ush."""
    U = len(v)
    smin, smax = v.min(), v.max()
    r = smax - smin
    delta = np.ldexp(r, -shift)
    c = delta - smin
    cform = (smin + c) >= 0.5 * delta
    x = v + c if cform else (v - smin) + delta
    xmin, xmax = (smin + c, smax + c) if cform else (delta, r + delta)
    b0, top = int(hi32(xmin)), int(hi32(xmax))
    span = top - b0 + 1
    scale = 0xFFFFFFFF if span <= MINBASE else int(MINBASE * 4294967296.0 / span) - 1
    key = ((hi32(x) - b0) * scale) >> 32
    ush = 0
    while ((U - 1) >> ush) >= MINSUB:
        ush += 1
    u = np.arange(U)
    return np.where(v == smin, MINBASE + (u >> ush), MINBASE - 1 - key)


def loop_cost(b, U):
    cnt = np.bincount(b, minlength=NB + 1)
    pos_b = np.sort(b)                 # bucket of each position
    size = cnt[pos_b]
    rows = (U + BLOCK - 1) // BLOCK
    per = rows * 64
    tot_valu = 0.0
    mx = []
    for wv in range(BLOCK // 64):
        for j in range(rows):
            a = wv * per + j * 64
            if a >= U:
                continue
            s = size[a:min(a + 64, U)]
            s = np.where(s > 1, s, 0)
            m = s.max()
            mx.append(m)
            tot_valu += 11 * (m // 2) + (8 if (s % 2).any() else 0)
    return np.mean(mx), tot_valu / (BLOCK // 64), (cnt > 0).sum(), cnt.max()


for name in ["combsum", "combmnz", "rrf", "wcombsum", "wcombmnz", "wrrf"]:
    ud, uc, perm, fz = co.fuse(off, docid, sc, R, name, 60, weights=w)
    st = []
    for q in range(Q):
        bq, U = off[q * R], uc[q]
        ranked = fz[bq:bq + U]
        v = np.empty(U)
        v[perm[bq:bq + U].astype(np.int64)] = ranked
        b = buckets(v)
        st.append((U,) + loop_cost(b, U))
    st = np.array(st, dtype=np.float64)
    print(f"{name:9s} U {st[:,0].mean():.0f}  max/wave-row {st[:,1].mean():.2f}  "
          f"loop VALU/wave {st[:,2].mean():.0f}  used buckets {st[:,3].mean():.0f}  biggest {st[:,4].mean():.1f}")
