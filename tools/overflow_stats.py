"""Bucket-overflow rate of qf_fuse's bucket sort on SURVEY §8(d)'s synthetic workload
(development; CPU only).  python tools/overflow_stats.py [n_queries] > profiles/...

The runs of the bench's default generator (oracle/synth_oracle.c, bit-identical to
qf_synth_runs_nq), per-query min-max to "%.6f" micro-units, the W-* weights from the
RSD column (min-max over the batch, "%.6f"), the six fusions by the C oracle; then, per
(query, method) pair, bsort_fast_kernel's keys restated (bs_key2: delta = range / 2^8,
mul_hi buckets over MINBASE, the minimum's sub-buckets by u; 2^12 buckets up to a union
of 3,072, 2^13 above): the largest bucket, whether it exceeds kJsBucketMax (128: the
recount with delta = range / 2^20), whether the recount still does (the fallback pass
sorts the pair), and the rank loop's work (sum of squared bucket sizes / U: compares
per item).
"""
import json
import math
import struct
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "qpp-fusion-rag_amd")]
from oracle import _loader as coracle  # noqa: E402

METHODS = ["combsum", "combmnz", "rrf", "wcombsum", "wcombmnz", "wrrf"]
BUCKET_MAX = 128


def hi32(x: np.ndarray) -> np.ndarray:
    return (np.ascontiguousarray(x, np.float64).view(np.uint64) >> np.uint64(32)).astype(np.uint64)


def key_consts(smin, smax, shift, minbase):
    """qf_fuse.hip bs_key2: (c, top, scale, cform) or None (the fallback pass)."""
    rng = smax - smin
    delta = math.ldexp(rng, -shift)
    if not (math.isfinite(rng) and delta > 0.0):
        return None
    c = delta - smin
    cform = math.isfinite(c) and (smin + c) >= 0.5 * delta
    xmin = smin + c if cform else delta
    xmax = smax + c if cform else rng + delta
    h = lambda x: struct.unpack("<Q", struct.pack("<d", x))[0] >> 32
    b0, top = h(xmin), h(xmax)
    span = (top - b0 + 1) & 0xFFFFFFFF
    scale = 0xFFFFFFFF if span <= minbase else int(minbase * 4294967296.0 / span) - 1
    return (c if cform else delta), top, scale, cform


def buckets(v, shift):
    U = len(v)
    bits = 12 if U <= 3072 else 13
    nb = 1 << bits
    minsub = nb // 16
    minbase = nb - minsub
    smin, smax = float(v.min()) + 0.0, float(v.max()) + 0.0
    if smin == smax:
        return None, nb
    k = key_consts(smin, smax, shift, minbase)
    if k is None:
        return "mark", nb
    c, top, scale, cform = k
    x = v + c if cform else (v - smin) + c
    key = ((np.uint64(top) - hi32(x)) & np.uint64(0xFFFFFFFF)) * np.uint64(scale) >> np.uint64(32)
    ush = 0
    while ((U - 1) >> ush) >= minsub:
        ush += 1
    u = np.arange(U, dtype=np.uint64)
    b = np.where(v == smin, np.uint64(minbase) + (u >> np.uint64(ush)), key)
    return np.bincount(b.astype(np.int64), minlength=nb), nb


def main():
    Q = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    R, K = 5, 1000
    import bench
    qo, qd = bench.nq_qrels()
    off, doc, raw = coracle.synth_runs_nq(0, Q, R, K, 20251212, qo, qd)
    norm = coracle.minmax_per_query(raw, off)
    micro = np.floor(norm * 1e6 + 0.5) / 1e6
    # RSD weights: raw column 5 of each list's top-100 (first 50), min-max per retriever
    cut = [raw[off[l]:off[l + 1]][:100] for l in range(Q * R)]
    coff = np.cumsum([0] + [len(c) for c in cut]).astype(np.int64)
    nt, tf = bench.text_inputs(0, Q)
    qraw = coracle.qpp_raw(np.concatenate(cut), coff, np.repeat(nt, R), np.repeat(tf[:, 0], R),
                           np.repeat(tf[:, 1], R))
    w = np.zeros(Q * R)
    for r in range(R):
        col = qraw[r::R, 5]
        lo, hi = col.min(), col.max()
        w[r::R] = np.floor((col - lo) / (hi - lo if hi > lo else 1.0) * 1e6 + 0.5) / 1e6
    out = {"generator": "nq (SURVEY 8(d), oracle/synth_oracle.c)", "queries": Q,
           "bucket_max": BUCKET_MAX, "methods": {}}
    for m in METHODS:
        _, uc, _, fused = coracle.fuse(off, doc, micro, R, m, 60,
                                       weights=w if m.startswith("w") else None)
        first, recount, fallback, mark, equal = 0, 0, 0, 0, 0
        work, largest = [], 0
        for q in range(Q):
            b, U = off[q * R], int(uc[q])
            v = fused[b:b + U]
            cnt, _ = buckets(v, 8)
            if cnt is None:
                equal += 1
                continue
            if isinstance(cnt, str):
                mark += 1
                continue
            largest = max(largest, int(cnt.max()))
            work.append(float((cnt.astype(np.float64) ** 2).sum() / U))
            if cnt.max() > BUCKET_MAX:
                first += 1
                cnt2, _ = buckets(v, 20)
                if isinstance(cnt2, str) or cnt2 is None or cnt2.max() > BUCKET_MAX:
                    fallback += 1
                else:
                    recount += 1
        out["methods"][m] = {
            "pairs": Q, "union_mean": float(uc.mean()), "union_max": int(uc.max()),
            "overflow_first_count": first, "sorted_after_recount": recount,
            "fallback_pass": fallback + mark, "all_equal": equal,
            "largest_bucket": largest, "rank_compares_per_item_mean": float(np.mean(work))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
