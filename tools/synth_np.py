"""numpy restatement of qf_synth_runs (csrc/qf_norm.hip synth_kernel) for offline
studies (development): the same docids; scores equal up to the device exp's last ulp."""
import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
PROFILES = [(0.50, 0.40, 2.0), (5.0, 25.0, 4.0), (-12.0, 11.5, 3.0), (60.0, 20.0, 2.5),
            (8.0, 30.0, 3.5), (1.0, 2.0, 3.0), (0.0, 1.0, 2.0), (-1.0, 3.0, 3.0)]


def mix64(z):
    z = np.asarray(z, np.uint64)
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def hash4(seed, a, b, c):
    u = np.uint64
    return mix64(u(seed) ^ mix64(np.asarray(a, u) ^ mix64(np.asarray(b, u) ^ mix64(np.asarray(c, u)))))


def u01(h):
    return (np.asarray(h, np.uint64) >> np.uint64(11)).astype(np.float64) * 2.0 ** -53


def synth(q_begin, n_q, R, K, seed=20251212, p_shared=0.7):
    off = np.arange(n_q * R + 1, dtype=np.int64) * K
    docid = np.empty(n_q * R * K, np.uint32)
    score = np.empty(n_q * R * K, np.float64)
    i = np.arange(K, dtype=np.uint64)
    for lq in range(n_q * R):
        r, qg = lq % R, q_begin + lq // R
        hl = int(hash4(seed, qg, r, 0xA11CE))
        he = hash4(seed, qg, r, i + np.uint64(1))
        shared = u01(he) < p_shared
        P = K
        A = (hl % P) | 1
        while A > 1:
            x, y = A, P
            while y:
                x, y = y, x % y
            if x == 1:
                break
            A += 2
            if A >= P:
                A = 1
        B = ((hl >> 32) % 3) if ((hl >> 20) & 1) else ((hl >> 32) % P)
        pidx = (A * i.astype(np.int64) + B) % P
        d_sh = ((qg * P + pidx) & 0x7FFFFFFF).astype(np.uint32)
        hq = int(hash4(seed, qg, 0xD0C, 0))
        base = (hq + r * K) % 0x7FFFFFFF
        d_un = (0x80000000 | ((base + i.astype(np.int64)) % 0x7FFFFFFF)).astype(np.uint32)
        sl = slice(lq * K, (lq + 1) * K)
        docid[sl] = np.where(shared, d_sh, d_un)
        A_, B_, c_ = PROFILES[r & 7]
        jitter = 0.8 + 0.4 * float(u01(hash4(seed, qg, r, 0x5CA1E)))
        t = (i.astype(np.float64) + 0.5 * u01(mix64(he))) / K
        score[sl] = A_ + B_ * jitter * np.exp(-c_ * t)
    return off, docid, score
