"""Native run-file I/O (libqfio.so, csrc/qf_io.cpp) vs pandas / Python (CPU).

The parser must produce exactly what read_csv + qppfuse.runset.pack_frames
produce, and the writer exactly the bytes of write_runfile's f-strings
(src/fusion.py:480-492), including Python's "%.6f" rounding.
"""
import math
import os

from pathlib import Path

import numpy as np
import pandas as pd
import pytest

from qppfuse import fastio
from qppfuse.runset import pack_frames


ROOT = Path(__file__).resolve().parents[1]

def _write_runs(tmp_path, rng, n_runs=4, n_q=30, k=50, text_fmt="%.6f"):
    names, paths = [], []
    for r in range(n_runs):
        name = f"Run{r}" if r != 2 else "BM25_MonoT5"
        lines = []
        for q in rng.permutation(n_q):  # queries interleaved in arbitrary file order
            qid = f"test{q}" if q % 5 else f"q{q:03d}"
            n = int(rng.integers(0, k))
            docs = rng.choice(5 * k, size=n, replace=False)
            sc = np.sort(rng.standard_normal(n) * 3)[::-1]
            if r == 1:
                sc = np.round(sc * 2) / 2  # ties
            for i, (d, s) in enumerate(zip(docs, sc)):
                docno = f"doc{d}" if d % 7 else f"Δ{d}"  # non-ASCII docnos
                lines.append(f"{qid}\tQ0 {docno}  {i + 1} {text_fmt % s} tag{r}\n")
        if r == 3:
            lines.insert(3, "\n")  # a blank line
        p = tmp_path / f"{name}.norm.res"
        p.write_text("".join(lines))
        names.append(name)
        paths.append(str(p))
    return names, paths


def _pandas_frames(paths, names):
    out = {}
    for p, n in zip(paths, names):
        df = pd.read_csv(p, sep=r"\s+", names=["qid", "iter", "docno", "rank", "score", "runid"],
                         dtype={"qid": str, "docno": str})
        df["qid"] = df["qid"].astype(str)
        out[n] = df
    return out


@pytest.mark.parametrize("fmt", ["%.6f", "%.9g"])
def test_parse_matches_pandas_and_pack(tmp_path, fmt):
    rng = np.random.default_rng(1)
    names, paths = _write_runs(tmp_path, rng, text_fmt=fmt)
    rs, frames = fastio.parse_runs(paths, names, n_threads=3)
    pf = _pandas_frames(paths, names)
    ref = pack_frames(pf)
    assert rs.qids == ref.qids and rs.rankers == ref.rankers
    assert list(rs.docnos) == list(ref.docnos)
    np.testing.assert_array_equal(rs.list_off, ref.list_off)
    np.testing.assert_array_equal(rs.docid, ref.docid)
    assert rs.score.tobytes() == ref.score.tobytes()
    np.testing.assert_array_equal(rs.rank, ref.rank)
    assert rs.canonical == ref.canonical and rs.rank_is_position == ref.rank_is_position
    assert (rs.micro is None) == (ref.micro is None)
    if rs.micro is not None:
        np.testing.assert_array_equal(rs.micro, ref.micro)
    for n in names:
        a, b = frames[n], pf[n]
        assert list(a.columns) == list(b.columns)
        for c in ("qid", "iter", "docno", "runid"):
            assert a[c].astype(str).tolist() == b[c].astype(str).tolist()
        np.testing.assert_array_equal(a["rank"].to_numpy(), b["rank"].to_numpy())
        assert a["score"].to_numpy().tobytes() == b["score"].to_numpy().tobytes()


def test_micro_units_when_every_score_is_six_decimal_text(tmp_path):
    p = tmp_path / "a.res"
    p.write_text("q1 Q0 d1 1 0.123456 t\nq1 Q0 d2 2 -3 t\nq2 Q0 d1 1 12.5 t\n")
    rs, _ = fastio.parse_runs([str(p)], ["a"])
    assert rs.micro.tolist() == [123456, -3000000, 12500000]
    p.write_text("q1 Q0 d1 1 0.000000 t\nq1 Q0 d2 2 -0.000000 t\n")  # -0.0 is no micro-unit
    rs, _ = fastio.parse_runs([str(p)], ["a"])
    assert rs.micro is None and math.copysign(1, rs.score[1]) < 0


def test_threads_do_not_change_the_result(tmp_path):
    rng = np.random.default_rng(2)
    names, paths = _write_runs(tmp_path, rng, n_q=80)
    a, _ = fastio.parse_runs(paths, names, n_threads=1)
    b, _ = fastio.parse_runs(paths, names, n_threads=8)
    np.testing.assert_array_equal(a.docid, b.docid)
    np.testing.assert_array_equal(a.list_off, b.list_off)


@pytest.mark.parametrize("threads", [1, 5])
def test_docnos_sharing_their_first_16_bytes(tmp_path, threads):
    """The interning recognises a repeat from (hash, length, first 16 bytes) and
    compares only the bytes past 16 for longer strings: docnos of 15-40 bytes that
    share 16-byte prefixes, differ in one late byte or only in length, and repeat
    across runs and queries must intern exactly as pack_frames does."""
    rng = np.random.default_rng(7)
    pre = ["abcdefghijklmnop", "abcdefghijklmnoq", "abcdefghijklmno"]
    pool = []
    for a in pre:
        pool += [a, a + "x", a + "xy", a + "y"]
        pool += [a + f"-{i:020d}" for i in range(40)]
        pool += [a + f"-{i:020d}z" for i in range(0, 40, 3)]
    names, paths = [], []
    for r in range(3):
        lines = []
        for q in range(25):
            docs = rng.choice(len(pool), size=int(rng.integers(1, 60)), replace=False)
            for i, d in enumerate(docs):
                lines.append(f"q{q} Q0 {pool[d]} {i + 1} {1.0 - i / 100:.6f} t{r}\n")
        pth = tmp_path / f"R{r}.norm.res"
        pth.write_text("".join(lines))
        names.append(f"R{r}")
        paths.append(str(pth))
    rs, _ = fastio.parse_runs(paths, names, n_threads=threads)
    ref = pack_frames(_pandas_frames(paths, names))
    assert list(rs.docnos) == list(ref.docnos)
    np.testing.assert_array_equal(rs.docid, ref.docid)
    np.testing.assert_array_equal(rs.list_off, ref.list_off)


def test_parse_errors(tmp_path):
    p = tmp_path / "bad.res"
    p.write_text("q1 Q0 d1 1 0.5 t\nq1 Q0 d2 2 t\n")
    with pytest.raises(ValueError, match="6 fields"):
        fastio.parse_runs([str(p)], ["bad"])
    with pytest.raises(FileNotFoundError):
        fastio.parse_runs([str(tmp_path / "missing.res")], ["m"])


def test_format_score_is_pythons_percent_6f():
    rng = np.random.default_rng(3)
    vals = list(rng.standard_normal(20000) * 10.0 ** rng.integers(-8, 9, 20000))
    vals += [k / 128 for k in range(-300, 300)]            # exact decimal ties
    vals += [(2 * k + 1) / 2e6 for k in range(-500, 500)]  # near ties
    vals += [0.0, -0.0, -1e-9, 1e-9, -4.9999999e-7, 5e-7, 2.0 ** 33, -(2.0 ** 33) - 0.5,
             1e15 + 0.125, 1.7976931348623157e308, 5e-324, math.inf, -math.inf, math.nan]
    for x in vals:
        assert fastio.format_score(x) == f"{x:.6f}", repr(x)


def test_write_run_matches_python_writer(tmp_path):
    from qppfuse.runset import RunSet
    rng = np.random.default_rng(4)
    Q, U = 25, 40
    qids = [f"test{i}" for i in range(Q)]
    docnos = np.array(sorted(f"d{i}" for i in range(300)), dtype=object)
    counts = rng.integers(0, U, Q).astype(np.int32)
    counts[3] = 0
    qbase = np.arange(Q, dtype=np.int64) * U
    ud = np.zeros(Q * U, np.uint32)
    perm = np.zeros(Q * U, np.uint16)
    fused = np.zeros(Q * U)
    for q in range(Q):
        n = counts[q]
        ud[q * U:q * U + n] = rng.choice(300, n, replace=False)
        perm[q * U:q * U + n] = rng.permutation(n)
        fused[q * U:q * U + n] = np.sort(rng.standard_normal(n))[::-1]
    fused[5] = -0.0
    rs = RunSet(qids=qids, rankers=["a"], docnos=docnos, list_off=np.zeros(2, np.int64),
                docid=np.zeros(0, np.uint32), score=np.zeros(0), rank=np.zeros(0, np.int64))
    order = np.array(sorted(range(Q), key=lambda i: int(qids[i][4:])), np.int64)
    out = tmp_path / "x.res"
    fastio.write_run(str(out), order, qbase, counts, ud, perm, fused, rs, "tag-1")
    want = []
    for q in order:
        for k in range(counts[q]):
            u = qbase[q] + perm[qbase[q] + k]  # qf_fuse's layout: scores by u, perm ranks
            want.append(f"{qids[q]} Q0 {docnos[ud[u]]} {k + 1} {fused[u]:.6f} tag-1\n")
    assert out.read_text() == "".join(want)
    # qf_fuse_wide's uint32 perm (qfio_write_run32): the same bytes
    out32 = tmp_path / "x32.res"
    fastio.write_run(str(out32), order, qbase, counts, ud, perm.astype(np.uint32), fused, rs,
                     "tag-1")
    assert out32.read_bytes() == out.read_bytes()
    # the chunked, pipelined writer (each chunk written once the one before it has
    # published its end): the same bytes over 1-8 threads, i.e. 8-64 chunks of 25
    # queries, over an existing longer file (truncated)
    out.write_text("x" * 100000)
    for threads in (1, 3, 8):
        fastio.write_run(str(out), order, qbase, counts, ud, perm, fused, rs, "tag-1",
                         n_threads=threads)
        assert out.read_text() == "".join(want), threads


def test_write_run_failure_leaves_existing_file(tmp_path):
    """A failed write (here: the target is a directory entry we cannot replace)
    leaves no temporary file behind and the old contents untouched."""
    from qppfuse.runset import RunSet
    rs = RunSet(qids=["q1"], rankers=["a"], docnos=np.array(["d0"], dtype=object),
                list_off=np.zeros(2, np.int64), docid=np.zeros(0, np.uint32),
                score=np.zeros(0), rank=np.zeros(0, np.int64))
    target = tmp_path / "busy"
    target.mkdir()  # rename(file, non-empty dir) fails
    (target / "keep").write_text("old")
    with pytest.raises(Exception):
        fastio.write_run(str(target), np.zeros(1, np.int64), np.zeros(1, np.int64),
                         np.array([1], np.int32), np.zeros(1, np.uint32), np.zeros(1, np.uint16),
                         np.ones(1), rs, "t")
    assert (target / "keep").read_text() == "old"
    assert sorted(p.name for p in tmp_path.iterdir()) == ["busy"]


def test_write_run_target_kinds(tmp_path):
    """The writer behaves like open(path, "w") for every kind of target:
    a symlink is written through (the link stays, its target gets the rows), an
    existing file keeps its mode, a new file gets 0666 & ~umask, /dev/null and a FIFO
    are written in place (the FIFO in order, read by another thread), and a writable
    file in a read-only directory is written in place; no temporary file is left."""
    import stat
    import threading
    from qppfuse.runset import RunSet
    rng = np.random.default_rng(11)
    Q, U = 40, 30
    qids = [f"test{i}" for i in range(Q)]
    docnos = np.array(sorted(f"d{i}" for i in range(200)), dtype=object)
    counts = np.full(Q, U, np.int32)
    qbase = np.arange(Q, dtype=np.int64) * U
    ud = np.concatenate([rng.choice(200, U, replace=False) for _ in range(Q)]).astype(np.uint32)
    perm = np.tile(np.arange(U, dtype=np.uint16), Q)
    fused = np.concatenate([np.sort(rng.random(U))[::-1] for _ in range(Q)])
    rs = RunSet(qids=qids, rankers=["a"], docnos=docnos, list_off=np.zeros(2, np.int64),
                docid=np.zeros(0, np.uint32), score=np.zeros(0), rank=np.zeros(0, np.int64))
    order = np.arange(Q, dtype=np.int64)
    want = "".join(f"{qids[q]} Q0 {docnos[ud[qbase[q] + k]]} {k + 1} {fused[qbase[q] + k]:.6f} t\n"
                   for q in range(Q) for k in range(U))
    write = lambda path, threads=4: fastio.write_run(str(path), order, qbase, counts, ud, perm,
                                                     fused, rs, "t", n_threads=threads)
    d = tmp_path / "d"
    d.mkdir()
    # a symlink: written through
    real = d / "real.res"
    real.write_text("old")
    link = d / "link.res"
    link.symlink_to(real)
    write(link)
    assert link.is_symlink() and real.read_text() == want
    # an existing file keeps its mode
    os.chmod(real, 0o640)
    write(real)
    assert stat.S_IMODE(real.stat().st_mode) == 0o640 and real.read_text() == want
    # a new file: 0666 & ~umask
    old = os.umask(0o027)
    try:
        write(d / "new.res")
    finally:
        os.umask(old)
    assert stat.S_IMODE((d / "new.res").stat().st_mode) == 0o640
    # /dev/null: no error, nothing replaced
    write("/dev/null")
    assert os.path.exists("/dev/null") and not os.path.isfile("/dev/null")
    # a FIFO: in order, in place
    fifo = d / "pipe"
    os.mkfifo(fifo)
    got = []
    reader = threading.Thread(target=lambda: got.append(open(fifo).read()))
    reader.start()
    write(fifo, threads=8)
    reader.join(60)
    assert got == [want] and stat.S_ISFIFO(os.stat(fifo).st_mode)
    # a writable file in a directory we cannot create files in: in place
    ro = tmp_path / "ro"
    ro.mkdir()
    f = ro / "x.res"
    f.write_text("old")
    os.chmod(ro, 0o555)
    try:
        write(f)  # (as root the mode is not enforced: then the rename path runs)
        assert f.read_text() == want
    finally:
        os.chmod(ro, 0o755)
    leftovers = [p.name for p in d.iterdir() if "qfio" in p.name] + \
        [p.name for p in ro.iterdir() if "qfio" in p.name]
    assert leftovers == []


@pytest.mark.parametrize("dtype,n", [(np.int32, 4 * 2**20 // 4 + 3), (np.int8, 4 * 2**20 + 9),
                                     (np.int8, 4 * 2**20 + 15), (np.float32, 2**20 + 7),
                                     (np.int16, 13), (np.int8, 1)])
def test_hash_bytes_tails(dtype, n):
    """Every tail length of the 16-byte loop (9-15 bytes overflowed an 8-byte word
    before round 4): the digest is deterministic and sees the last byte."""
    rng = np.random.default_rng(n)
    a = rng.integers(-100, 100, n).astype(dtype)
    h = fastio.hash_bytes(a)
    assert h == fastio.hash_bytes(a.copy())
    b = a.copy()
    b.view(np.uint8)[-1] ^= 0x5A
    assert fastio.hash_bytes(b) != h
    nbytes = a.nbytes
    tail = nbytes % 16
    for i in {nbytes - tail, nbytes - tail + 8} if tail > 8 else {nbytes - tail} if tail else ():
        c = a.copy()
        c.view(np.uint8)[i] ^= 1  # the first byte of each tail word
        assert fastio.hash_bytes(c) != h, i


def test_write_run_uint32_perm_beyond_65535():
    """A union of 70,000 documents: ranks past u = 65,535 through the uint32 perm."""
    import tempfile
    from qppfuse.runset import RunSet
    rng = np.random.default_rng(6)
    n = 70_000
    docnos = np.array([f"d{i:06d}" for i in range(n)], dtype=object)
    ud = rng.permutation(n).astype(np.uint32)
    fused = rng.standard_normal(n)
    perm = np.argsort(-fused, kind="stable").astype(np.uint32)
    rs = RunSet(qids=["q1"], rankers=["a"], docnos=docnos, list_off=np.zeros(2, np.int64),
                docid=np.zeros(0, np.uint32), score=np.zeros(0), rank=np.zeros(0, np.int64))
    with tempfile.TemporaryDirectory() as d:
        out = Path(d) / "w.res"
        fastio.write_run(str(out), np.zeros(1, np.int64), np.zeros(1, np.int64),
                         np.array([n], np.int32), ud, perm, fused, rs, "t")
        lines = out.read_text().splitlines()
    assert len(lines) == n
    for k in (0, 65535, 65536, n - 1):
        u = perm[k]
        assert lines[k] == f"q1 Q0 {docnos[ud[u]]} {k + 1} {fused[u]:.6f} t"


def test_load_runs_returns_frames_and_caches_the_pack(tmp_path):
    from qppfuse import fusion
    rng = np.random.default_rng(5)
    names, paths = _write_runs(tmp_path, rng)
    frames = fusion.load_runs(str(tmp_path))
    assert list(frames) == [f.replace(".norm.res", "") for f in os.listdir(tmp_path)
                            if f.endswith(".norm.res")]
    rs = fusion._pack(frames)
    assert rs.n_entries == sum(len(df) for df in frames.values())


@pytest.mark.parametrize("case", ["shifted_ranks", "unsorted_scores", "canonical"])
def test_list_flags_match_pack(tmp_path, case):
    """rank_is_position / canonical computed by the native loader == pack_frames'."""
    lines = []
    for q in range(4):
        for i in range(6):
            rank = i + (2 if case == "shifted_ranks" else 1)
            score = 1.0 - i / 10
            if case == "unsorted_scores" and q == 2 and i == 3:
                score = 0.95
            lines.append(f"{q} Q0 d{q}_{i} {rank} {score:.6f} t\n")
    p = tmp_path / "A.norm.res"
    p.write_text("".join(lines))
    rs, _ = fastio.parse_runs([str(p)], ["A"])
    ref = pack_frames(_pandas_frames([str(p)], ["A"]))
    assert (rs.rank_is_position, rs.canonical) == (ref.rank_is_position, ref.canonical)
    assert (rs.rank_is_position, rs.canonical) == {
        "shifted_ranks": (False, True), "unsorted_scores": (True, False),
        "canonical": (True, True)}[case]


@pytest.mark.parametrize("mode", ["arrow", "object"])
def test_frame_string_modes(tmp_path, monkeypatch, mode):
    """load_runs' string columns: Arrow-backed (default, no Python str per row) or
    object; both hold the values read_csv gives, and the run set is the same."""
    monkeypatch.setenv("QPPFUSE_FRAME_STRINGS", mode)
    rng = np.random.default_rng(3)
    names, paths = _write_runs(tmp_path, rng)
    rs, frames = fastio.parse_runs(paths, names, n_threads=4)
    pf = _pandas_frames(paths, names)
    for n in names:
        for c in ("qid", "iter", "docno", "runid"):
            col = frames[n][c]
            assert (str(col.dtype) == "string") if mode == "arrow" else (col.dtype == object)
            assert col.astype(str).tolist() == pf[n][c].astype(str).tolist()
    ref = pack_frames(pf)
    assert list(rs.docnos) == list(ref.docnos)


def test_gather_strings_matches_python():
    words = ["test0", "", "Δ17", "doc123456789", "x"]
    enc = [w.encode() for w in words]
    off = np.zeros(len(enc) + 1, np.int64)
    np.cumsum([len(e) for e in enc], out=off[1:])
    chars = np.frombuffer(b"".join(enc), np.uint8).copy()
    rng = np.random.default_rng(0)
    for n in (0, 1, 7, 1000, 200003):  # ragged thread ranges
        codes = rng.integers(0, len(words), n).astype(np.uint32)
        assert list(fastio.arrow_strings(off, chars, codes)) == [words[c] for c in codes]


def test_string_table_lookups():
    from qppfuse.runset import StringTable
    words = ["a", "bb", "Δc", "d"]
    enc = [w.encode() for w in words]
    off = np.zeros(5, np.int64)
    np.cumsum([len(e) for e in enc], out=off[1:])
    t = StringTable(off, b"".join(enc))
    assert len(t) == 4 and t[1] == "bb" and t[-1] == "d"
    with pytest.raises(IndexError):
        t[4]
    assert t[np.array([2, 0, 2])].tolist() == ["Δc", "a", "Δc"]
    assert list(t) == words and np.asarray(t, dtype=object).tolist() == words
    assert t[np.array([3, 1])].tolist() == ["d", "bb"]  # after materialisation too


def test_pack_cache_follows_edits_of_arrow_frames(tmp_path, monkeypatch):
    """load_runs' Arrow-backed frames: the cached run set is reused while the
    frames are unchanged and rebuilt after an edit of a string or numeric column."""
    from qppfuse import fusion
    monkeypatch.setenv("QPPFUSE_FRAME_STRINGS", "arrow")
    rng = np.random.default_rng(5)
    _write_runs(tmp_path, rng, n_runs=3, n_q=6, k=8)
    frames = fusion.load_runs(str(tmp_path))
    a = fusion._pack(frames)
    assert fusion._pack(frames) is a
    name = next(iter(frames))
    frames[name].loc[0, "docno"] = "zzz_new"
    b = fusion._pack(frames)
    assert b is not a and "zzz_new" in list(b.docnos)
    frames[name].loc[1, "score"] = 123.0
    c = fusion._pack(frames)
    assert c is not b and 123.0 in c.score
    assert fusion._pack(frames) is c


def test_parse_line_shapes_against_pandas(tmp_path):
    """Lines the SIMD field split does not take (>= 64 bytes, the mapping's last 64
    bytes) next to ones it does; CRLF, tab separators, no final newline,
    and a qid whose rows come in two separate runs of one file (its list keeps the
    file order of both runs)."""
    long_doc = "doc-" + "x" * 70
    rows_a = [
        "q1 Q0 d1 1 0.900000 A\r\n",
        f"q1 Q0 {long_doc} 2 0.800000 A\r\n",
        "q2\tQ0\td2 1 0.700000 A\n",
        "q1 Q0 d3 3 0.600000\tA\n",   # q1 again, after q2: a second run of q1
        "q2 Q0 d1 2 0.500000 A\n",
        f"q3 Q0 {long_doc}y 1 0.400000 A",  # no final newline
    ]
    rows_b = ["q2 Q0 d9 1 0.300000 B\n", "q1 Q0 d1 1 0.200000 B\n"]
    pa_, pb_ = tmp_path / "A.res", tmp_path / "B.res"
    pa_.write_text("".join(rows_a))
    pb_.write_text("".join(rows_b))
    paths, names = [str(pa_), str(pb_)], ["A", "B"]
    for threads in (1, 3):
        rs, frames = fastio.parse_runs(paths, names, n_threads=threads)
        pf = _pandas_frames(paths, names)
        ref = pack_frames(pf)
        assert rs.qids == ref.qids and list(rs.docnos) == list(ref.docnos)
        np.testing.assert_array_equal(rs.list_off, ref.list_off)
        np.testing.assert_array_equal(rs.docid, ref.docid)
        assert rs.score.tobytes() == ref.score.tobytes()
        np.testing.assert_array_equal(rs.rank, ref.rank)
        for n in names:
            for c in ("qid", "iter", "docno", "runid"):
                assert frames[n][c].astype(str).tolist() == pf[n][c].astype(str).tolist()


def _py_score_lists(path, top_k):
    """src/qpp.py:292-305 as the reference runs it."""
    from collections import defaultdict
    runs = defaultdict(list)
    with open(path, "r") as f:
        for line in f:
            parts = line.strip().split()
            if len(parts) >= 5:
                runs[parts[0]].append(float(parts[4]))
    return {q: sorted(v, reverse=True)[:top_k] for q, v in runs.items()}


def _native_as_dict(got):
    qids, off, sc = got[:3]
    return {q: sc[off[i]:off[i + 1]].tolist() for i, q in enumerate(qids)}


@pytest.mark.parametrize("top_k", [100, 3, 1, -2, 10**6])
@pytest.mark.parametrize("threads", [1, 3, 8])
def test_read_score_lists_matches_reference_loop(tmp_path, top_k, threads):
    rng = np.random.default_rng(7)
    lines = []
    qids = [f"q{i}" for i in rng.permutation(40)] + ["7", "test3", "10"]
    for rep in range(2):  # qids interleaved: a query's rows in two blocks
        for q in qids:
            for k in range(int(rng.integers(0, 30))):
                s = rng.choice([f"{rng.normal():.6f}", f"{rng.normal() * 1e5:.3e}", "0.0", "-0.0",
                                "-0", "+1.5", "1.", ".5", "inf", "-Infinity", "1E-3",
                                f"{rng.normal()!r}"])
                tail = rng.choice(["bm25", "bm25 extra fields", ""])
                lines.append(f"{q} Q0 d{k} {k + 1} {s} {tail}".rstrip())
        lines += ["", "   ", "short line", "a b c d"]  # < 5 fields: skipped
    p = tmp_path / "x.res"
    p.write_text("\r\n".join(lines[:len(lines) // 2]) + "\r\n" + "\n".join(lines[len(lines) // 2:]))
    want = _py_score_lists(p, top_k)
    got = fastio.read_score_lists(str(p), top_k, n_threads=threads)
    assert got is not None
    assert list(want) == got[0]  # first-appearance order
    g = _native_as_dict(got)
    for q in want:  # bit-exact, -0.0 / 0.0 positions included
        assert np.array(want[q]).tobytes() == np.array(g[q], np.float64).tobytes(), q
    assert got[3] == sum(1 for ln in p.read_text().splitlines() if len(ln.split()) >= 5)


@pytest.mark.parametrize("text", ["q1 Q0 d 1 0.5_1 t", "q1 Q0 d 1 nan t", "q1 Q0 dé 1 0.5 t",
                                  "q1 Q0 d 1 0.5 t\rq2 Q0 e 1 0.25 t", "q1\x1cQ0 d 1 0.5 t"])
def test_read_score_lists_defers_to_python(tmp_path, text):
    p = tmp_path / "x.res"
    p.write_text("q0 Q0 a 1 1.0 t\n" + text + "\n", newline="")
    assert fastio.read_score_lists(str(p), 100) is None


def test_read_score_lists_errors_like_float(tmp_path):
    p = tmp_path / "x.res"
    p.write_text("q0 Q0 a 1 1.0 t\nq0 Q0 b 2 0x1p3 t\n")
    with pytest.raises(ValueError, match="could not convert string to float: '0x1p3'"):
        fastio.read_score_lists(str(p), 100)
    with pytest.raises(ValueError):
        float("0x1p3")
    with pytest.raises(FileNotFoundError):
        fastio.read_score_lists(str(tmp_path / "missing.res"), 100)
    e = tmp_path / "empty.res"
    e.write_text("")
    got = fastio.read_score_lists(str(e), 100)
    assert got[0] == [] and got[1].tolist() == [0]


def test_rawarray_large_then_small_resize(tmp_path):
    """qf_io.cpp's RawArray mmaps buffers >= 4 MB and mallocs smaller ones; release()
    must forget the mapping, or a later small resize() would munmap a malloc'd
    pointer.  A C++ harness including the translation unit (g++, no
    GPU) resizes large -> small -> large -> small and frees each through the same
    release path; it runs under glibc's heap checks (MALLOC_CHECK_=3)."""
    import os
    import shutil
    import subprocess
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    src = tmp_path / "rawarray.cpp"
    src.write_text(
        '#include "%s"\n'
        "int main() {\n"
        "  RawArray<double> a;\n"
        "  for (int r = 0; r < 3; ++r) {\n"
        "    a.resize((8u << 20) / sizeof(double));  // mmap'd\n"
        "    if (!a.mapped) return 2;\n"
        "    a[0] = 1.0;\n"
        "    a.resize(16);                            // malloc'd\n"
        "    if (a.mapped) return 3;\n"
        "    a[15] = 2.0;\n"
        "  }\n"
        "  a.release();\n"
        "  if (a.mapped || a.data() != nullptr) return 4;\n"
        "  return 0;\n"
        "}\n" % (ROOT / "qpp-fusion-rag_amd" / "csrc" / "qf_io.cpp"))
    exe = tmp_path / "rawarray"
    subprocess.run([gxx, "-O1", "-std=c++17", "-fopenmp", "-o", str(exe), str(src)], check=True,
                   timeout=300)
    r = subprocess.run([str(exe)], env=dict(os.environ, MALLOC_CHECK_="3"), timeout=60)
    assert r.returncode == 0


@pytest.mark.parametrize("extra", ["", "q1 Q0 short 1\n", "q2 Q0 d7 3 0.5 tag more\n"])
def test_load_run_file_native_equals_the_reference_loop(tmp_path, extra):
    """data_utils.load_run_file parses with qfio and builds the reference's dict
    (src/data_utils.py:204-231: first-appearance query order, rows stably sorted by
    rank, float / int values); a file qfio rejects takes the reference's loop."""
    from qppfuse import data_utils as du
    rng = np.random.default_rng(3)
    lines = [f"q{rng.integers(0, 40)} Q0 d{rng.integers(0, 500)} {rng.integers(1, 60)} "
             f"{rng.random() * 20:.6f} run\n" for _ in range(4000)]
    lines += ["q3 Q0 dX 7 1e-7 run\n", "q9 Q0 dY 2 -3.25 tagg\n", "q9 Q0 dZ 2 21.35099 tagg\n"]
    p = tmp_path / "run.res"
    p.write_text("".join(lines) + extra)
    got = du.load_run_file(p)
    want = du._load_run_file_lines(p)
    assert list(got) == list(want)
    assert got == want


def test_load_run_file_grouped_file_equals_the_reference_loop(tmp_path):
    """A file already grouped by query in rank order (ties included) takes
    load_run_file's no-sort branch: the same dict as the reference's loop."""
    from qppfuse import data_utils as du
    rng = np.random.default_rng(8)
    lines = []
    for q in rng.permutation(30):
        ranks = np.sort(rng.integers(1, 40, size=50))  # repeated ranks: stable ties
        lines += [f"q{q} Q0 d{rng.integers(0, 900)} {r} {rng.random():.6f} run\n" for r in ranks]
    p = tmp_path / "grouped.res"
    p.write_text("".join(lines))
    got = du.load_run_file(p)
    want = du._load_run_file_lines(p)
    assert list(got) == list(want)
    assert got == want
