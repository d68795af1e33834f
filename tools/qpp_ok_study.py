"""Can SigmaMax (col 3) and CumNQC (col 9) use O(k) prefix statistics and keep every
.qpp value?    CPU study, development only.

The reference computes each prefix's statistics from scratch (QPPBridge.java:269-293:
a compensated mean of the prefix, then the compensated mean of (x - mean)^2 over it;
:400-410: NQC of Arrays.copyOf(rsvs, k) for every k) — O(k^2) per list.  An O(k)
form carries running sums (Welford's mean / M2 update).  This script runs both over
C2-shaped synthetic lists (tools/synth_np.py, the device generator's numpy twin:
top-100 of each 1000-entry list, as compute_qpp_for_res_file cuts it) and compares:
the raw predictors (relative difference), and what reaches the fusion — the per-file
min-max normalised value written "%.6f" (src/qpp.py:340-374, 329-335).
python tools/qpp_ok_study.py [n_queries]
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tools")]
from oracle import _loader as coracle  # noqa: E402
from synth_np import synth  # noqa: E402


def f32(x):
    return np.asarray(x, np.float64).astype(np.float32).astype(np.float64)


def welford_prefix(x):
    """[k] population variances of the prefixes x[:i+1] by Welford's update (O(k))."""
    mean, m2 = 0.0, 0.0
    out = np.zeros(len(x))
    for i, v in enumerate(x):
        d = v - mean
        mean += d / (i + 1)
        m2 += d * (v - mean)
        out[i] = m2 / (i + 1)
    return out


def ok_cols(x, num_terms):
    """SigmaMax and CumNQC from the O(k) prefix variances (k = min(50, n))."""
    n = len(x)
    if n < 2:
        return 0.0, 0.0
    var = welford_prefix(x)
    sigma_max = float(np.max(np.sqrt(np.maximum(var[1:], 0.0)))) / np.sqrt(max(1, num_terms))
    cum = float(np.sum(var[1:])) / (n - 1)
    return sigma_max, cum


def main():
    Q = int(sys.argv[1]) if len(sys.argv) > 1 else 3452
    R, K = 5, 1000
    off, _, raw = synth(0, Q, R, K)
    rng = np.random.default_rng(3)
    nt = rng.integers(2, 15, Q).astype(np.int32)
    # compute_qpp_for_res_file's lists: sorted desc, [:100]; Java: float32, first 50
    lists = [np.sort(raw[off[l]:off[l + 1]])[::-1][:100] for l in range(Q * R)]
    cut = np.zeros(Q * R + 1, np.int64)
    cut[1:] = np.cumsum([len(x) for x in lists])
    exact = coracle.qpp_raw(np.concatenate(lists), cut, np.repeat(nt, R), np.zeros(Q * R),
                            np.zeros(Q * R))
    ok = exact.copy()
    for l, x in enumerate(lists):
        ok[l, 3], ok[l, 9] = ok_cols(f32(x[:50]), int(nt[l // R]))
    rel = np.abs(ok - exact) / np.maximum(np.abs(exact), 1e-300)
    res = {"queries": Q, "lists": Q * R,
           "raw_bit_identical": {c: int(np.sum(ok[:, c] == exact[:, c])) for c in (3, 9)},
           "raw_max_rel_diff": {c: float(rel[:, c].max()) for c in (3, 9)}}
    # per retriever file: min-max over its queries, then "%.6f"
    diff6 = {3: 0, 9: 0}
    for r in range(R):
        for c in (3, 9):
            for arr_name, arr in (("e", exact), ("o", ok)):
                pass
            e, o = exact[r::R, c], ok[r::R, c]
            ne = (e - e.min()) / (e.max() - e.min() if e.max() > e.min() else 1.0)
            no = (o - o.min()) / (o.max() - o.min() if o.max() > o.min() else 1.0)
            diff6[c] += int(sum(f"{a:.6f}" != f"{b:.6f}" for a, b in zip(ne, no)))
    res["qpp_text_values_changed"] = diff6
    res["qpp_text_values_per_column"] = Q * R
    print(json.dumps(res))


if __name__ == "__main__":
    main()
