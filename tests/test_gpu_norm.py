"""Per-query min-max normalisation kernel vs the oracle — needs an MI355X."""
import numpy as np
import pytest
import torch

from oracle import _loader as coracle
from tests.helpers import unhex

pytestmark = pytest.mark.gpu


def test_minmax_bit_exact_and_micro_is_python_format(gpu):
    from qppfuse import engine
    rng = np.random.default_rng(1)
    lens = rng.integers(0, 1500, 400)
    lens[:3] = [1, 2, 0]
    lists = [np.sort(rng.normal(0, 10, n))[::-1] for n in lens]
    lists[10] = np.full(17, 4.25)  # constant list -> all zeros
    off = np.cumsum([0] + [len(l) for l in lists]).astype(np.int64)
    flat = np.concatenate(lists)
    norm, micro = engine.minmax_per_query(torch.from_numpy(flat).to(gpu),
                                          torch.from_numpy(off).to(gpu))
    norm, micro = norm.cpu().numpy(), micro.cpu().numpy()
    want = coracle.minmax_per_query(flat, off)
    assert norm.tobytes() == want.tobytes()
    fmt = [f"{v:.6f}" for v in want]
    got = [f"{m // 10**6}.{m % 10**6:06d}" for m in micro]
    assert got == fmt


@pytest.mark.parametrize("n_lists", [1, 7, 32768, 32769])
def test_minmax_batch_sizes_and_list_lengths(gpu, n_lists):
    """One to 32,769 lists of 0-1,100 entries (the 4-row register body up to 256, the
    16-row one up to 1,024, the loop beyond, and each boundary), odd counts:
    bit-exact, and the micro-units are "%.6f"."""
    from qppfuse import engine
    rng = np.random.default_rng(n_lists)
    lens = rng.integers(0, 80, n_lists)
    lens[rng.random(n_lists) < 0.05] = 512
    lens[rng.random(n_lists) < 0.02] = 513
    lens[rng.random(n_lists) < 0.01] = 1100
    edge = [256, 257, 255, 1024, 1025, 100, 64, 65]
    lens[:min(len(edge), n_lists)] = edge[:n_lists]
    off = np.cumsum(np.concatenate([[0], lens])).astype(np.int64)
    flat = np.repeat(rng.normal(0, 5, n_lists), lens) + rng.random(int(off[-1]))
    norm, micro = engine.minmax_per_query(torch.from_numpy(flat).to(gpu),
                                          torch.from_numpy(off).to(gpu))
    want = coracle.minmax_per_query(flat, off)
    assert norm.cpu().numpy().tobytes() == want.tobytes()
    m = micro.cpu().numpy()
    assert [f"{x // 10**6}.{x % 10**6:06d}" for x in m] == [f"{v:.6f}" for v in want]


def test_round6_half_even_and_hard_cases(gpu):
    """Values next to 6th-decimal ties: the exact binary value decides (CPython)."""
    from qppfuse import engine
    base = np.array([0.0000005, 0.0000015, 0.0000025, 0.1234565, 0.9999995, 0.5, 1.0,
                     0.3333335, 0.0000004999999, 0.7654325])
    vals = np.concatenate([base, np.nextafter(base, 2), np.nextafter(base, -1)])
    vals = np.clip(vals, 0, 1)
    rng = np.random.default_rng(5)
    vals = np.concatenate([vals, rng.random(100_000),
                           np.round(rng.random(20_000), 7)])
    # one list [1, vals..., 0] so min-max is the identity
    flat = np.concatenate([[1.0], np.sort(vals)[::-1], [0.0]])
    off = np.array([0, len(flat)], np.int64)
    _, micro = engine.minmax_per_query(torch.from_numpy(flat).to(gpu),
                                       torch.from_numpy(off).to(gpu))
    micro = micro.cpu().numpy()
    got = [f"{m // 10**6}.{m % 10**6:06d}" for m in micro]
    assert got == [f"{v:.6f}" for v in flat]


def test_normalize_scores_matches_reference_golden(gpu, golden):
    from qppfuse.retrieval import normalize_scores
    for case in golden["normalize_scores"]:
        src = [(d, unhex(s), r) for d, s, r in case["in"]]
        want = [(d, unhex(s), r) for d, s, r in case["out"]]
        assert normalize_scores(src) == want


def test_write_run_reference_drop_in(gpu, golden3, tmp_path):
    """scripts/02_retrieve.py:65-82 as the reference calls it: {qid: RetrieverResult}
    into a directory that does not exist yet; bytes == the reference's own output
    (tests/golden/make_golden.py round3: base.py's RetrieverResult + normalize_scores)."""
    from qppfuse.retrieval import RetrieverResult, write_run
    for i, case in enumerate(golden3["write_run"]):
        res = {q: RetrieverResult(qid=q, results=[(d, unhex(s), r) for d, s, r in docs],
                                  retriever_name=case["retriever_name"])
               for q, docs in case["results"].items()}
        p = tmp_path / f"c{i}" / "runs" / "nested" / "X.res"
        write_run(res, str(p), case["retriever_name"], normalize=case["normalize"])
        assert p.read_text() == case["expected"], (case["kind"], case["normalize"])


def test_write_run_normalized_text(gpu, tmp_path):
    from qppfuse.retrieval import RetrieverResult, write_run
    rng = np.random.default_rng(2)
    results = {f"test{i}": [(f"d{j}", float(s), j + 1) for j, s in
                            enumerate(sorted(rng.gamma(2, 6, 20), reverse=True))]
               for i in range(12)}
    p = tmp_path / "X.norm.res"
    write_run({q: RetrieverResult(q, d, "X") for q, d in results.items()}, str(p), "X",
              normalize=True)
    from oracle import ref_port
    want = []
    for qid in sorted(results, key=ref_port.qid_sort_key):
        for d, s, r in ref_port.normalize_scores(results[qid]):
            want.append(f"{qid} Q0 {d} {r} {s:.6f} X\n")
    assert p.read_text() == "".join(want)
