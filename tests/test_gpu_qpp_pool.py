"""scripts/03_qpp.py's fan-out (scripts/03_qpp.py:92-130) over the drop-in.

The reference's 03_qpp imports compute_qpp_for_res_file in the parent (which
never touches a device), then runs it for every raw .res file in a
ProcessPoolExecutor (fork on Linux): each worker opens its own HIP context.
The .qpp files the workers write must equal, byte for byte, the ones one
process writes, and match the CPU restatement of the reference pipeline.
"""
import subprocess
import sys
import textwrap
from pathlib import Path

import numpy as np
import pytest

from oracle import ref_port

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu

SCRIPT = textwrap.dedent('''
    import os, sys
    sys.path[:0] = [{root!r}, {pkg!r}]
    from concurrent.futures import ProcessPoolExecutor, as_completed
    from qppfuse import compute_qpp_for_res_file   # the parent touches no device

    def _process_qpp_file(args_tuple):  # scripts/03_qpp.py:31-36
        res_path, qpp_output, top_k, normalize, queries_path, res_file = args_tuple
        compute_qpp_for_res_file(res_path, qpp_output, top_k, normalize, queries_path)
        return res_file

    if __name__ == "__main__":
        runs_dir, qpp_dir, queries = sys.argv[1:4]
        res_files = [f for f in os.listdir(runs_dir)
                     if f.endswith(".res") and not f.endswith(".norm.res")]
        jobs = [(os.path.join(runs_dir, f), os.path.join(qpp_dir, f.replace(".res", ".res.mmnorm.qpp")),
                 100, "minmax", queries, f) for f in res_files]
        assert "torch" not in sys.modules or not __import__("torch").cuda.is_initialized()
        done = []
        with ProcessPoolExecutor(max_workers=min(8, len(jobs))) as ex:
            futures = {{ex.submit(_process_qpp_file, j): j for j in jobs}}
            for fut in as_completed(futures):
                done.append(fut.result())   # a worker's exception fails the run
        assert "torch" not in sys.modules or not __import__("torch").cuda.is_initialized()
        print("done", sorted(done))
''')


def _write_runs(d: Path, rng):
    """Three raw runs (file order shuffled, BM25-like / dense-like / negative scores)."""
    import json
    texts = {}
    with open(d / "queries.jsonl", "w") as fq:
        for qi in range(150):
            qid = f"test{qi}"  # one kind: the .qpp writer's sort key rejects mixed ones
            texts[qid] = " ".join(f"w{j}" * (j % 4 + 1) for j in range(qi % 9 + 1))
            fq.write(json.dumps({"_id": qid, "text": texts[qid]}) + "\n")
    runs = d / "runs"
    runs.mkdir()
    gens = {"BM25": lambda n: rng.gamma(2, 6, n) + 5, "BGE": lambda n: 0.5 + 0.4 * rng.beta(5, 2, n),
            "MonoT5": lambda n: -rng.gamma(2, 2, n)}
    for name, g in gens.items():
        rows = []
        for qid in texts:
            sc = g(int(rng.integers(1, 400)))
            for rank, s in enumerate(sorted(sc, reverse=True), 1):
                rows.append(f"{qid} Q0 d{rank}x{qid} {rank} {float(s)!r} {name}\n")
        rng.shuffle(rows)
        (runs / f"{name}.res").write_text("".join(rows))
        (runs / f"{name}.norm.res").write_text("")  # 03_qpp skips .norm.res
    return runs, texts


def test_03_qpp_process_pool_matches_single_process(gpu, tmp_path):
    from qppfuse import textfeat
    from qppfuse.qpp import compute_qpp_for_res_file
    rng = np.random.default_rng(33)
    runs, texts = _write_runs(tmp_path, rng)
    pool_dir = tmp_path / "qpp_pool"
    pool_dir.mkdir()
    script = tmp_path / "qpp03.py"
    script.write_text(SCRIPT.format(root=str(ROOT), pkg=str(ROOT / "qpp-fusion-rag_amd")))
    r = subprocess.run([sys.executable, str(script), str(runs), str(pool_dir),
                        str(tmp_path / "queries.jsonl")], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "done ['BGE.res', 'BM25.res', 'MonoT5.res']" in r.stdout
    for name in ("BGE", "BM25", "MonoT5"):
        one = tmp_path / f"{name}.one.qpp"
        got = compute_qpp_for_res_file(str(runs / f"{name}.res"), str(one), 100, "minmax",
                                       str(tmp_path / "queries.jsonl"))
        pooled = pool_dir / f"{name}.res.mmnorm.qpp"
        assert pooled.read_bytes() == one.read_bytes(), name
        # and the restated reference pipeline (src/qpp.py:291-337, QPPBridge restated)
        per_q = {}
        for line in (runs / f"{name}.res").read_text().splitlines():
            f = line.split()
            per_q.setdefault(f[0], []).append(float(f[4]))
        raw = {}
        for q, s in per_q.items():
            nt, mi, ai = textfeat.features(texts[q])
            d = ref_port.java_qpp(nt, mi, ai, sorted(s, reverse=True)[:100])
            raw[q] = [d[n] for n in ref_port.QPP_NAMES]
        want = ref_port.normalize_qpp(raw, "minmax")
        assert list(got) == list(want)
        for q in want:
            np.testing.assert_allclose(got[q], want[q], rtol=1e-7, atol=1e-9)
