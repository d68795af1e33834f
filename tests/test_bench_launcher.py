"""bench.py's multi-GPU entry (CPU): `--gpus N` without a launcher starts N ranks.

The driver runs `torch.distributed.run --nproc-per-node N bench.py --gpus N`;
a plain `python bench.py --gpus N` must do the same by itself (one process
per GPU, rendezvous on 127.0.0.1) before any GPU call, and a WORLD_SIZE that
disagrees with --gpus is refused.  The rank processes here run a stand-in
script (the real bench needs a GPU) through the same launcher code.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _bench():
    sys.path.insert(0, str(ROOT))
    import bench
    return bench


def test_launcher_starts_n_ranks(tmp_path, monkeypatch):
    bench = _bench()
    script = tmp_path / "rank.py"
    out = tmp_path / "ranks"
    out.mkdir()
    script.write_text(
        "import os, json, sys\n"
        f"d = {str(out)!r}\n"
        "r = os.environ['RANK']\n"
        "json.dump({k: os.environ.get(k) for k in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK',"
        " 'MASTER_ADDR', 'QPPFUSE_BENCH_LAUNCHED')} | {'argv': sys.argv[1:]},"
        " open(os.path.join(d, r + '.json'), 'w'))\n")
    args = type("A", (), {"gpus": 3})()
    rc = bench.launch_ranks(args, script=script, argv=["--gpus", "3", "--steps", "2"])
    assert rc == 0
    got = sorted(json.loads(p.read_text())["RANK"] for p in out.iterdir())
    assert got == ["0", "1", "2"]
    one = json.loads((out / "1.json").read_text())
    assert one["WORLD_SIZE"] == "3" and one["MASTER_ADDR"] == "127.0.0.1"
    assert one["QPPFUSE_BENCH_LAUNCHED"] == "1"
    assert one["argv"] == ["--gpus", "3", "--steps", "2"]


def test_launcher_propagates_failure(tmp_path):
    bench = _bench()
    script = tmp_path / "fail.py"
    script.write_text("import os, sys\nsys.exit(3 if os.environ['RANK'] == '1' else 0)\n")
    args = type("A", (), {"gpus": 2})()
    assert bench.launch_ranks(args, script=script, argv=[]) != 0


def test_world_size_must_match_gpus(monkeypatch):
    bench = _bench()
    monkeypatch.setenv("WORLD_SIZE", "2")
    args = type("A", (), {"gpus": 4, "rehearse_one_gpu": False, "dist_backend": "gloo"})()
    with pytest.raises(SystemExit, match="--gpus 4 but WORLD_SIZE=2"):
        bench.setup_dist(args)


def test_main_dispatches_to_launcher_before_gpu(monkeypatch):
    """`python bench.py --gpus 2` (no WORLD_SIZE): main() hands over to the launcher
    and exits with its code without touching torch.cuda."""
    bench = _bench()
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "1"])
    seen = {}

    def fake(args, script=None, argv=None):
        seen["gpus"] = args.gpus
        return 7
    monkeypatch.setattr(bench, "launch_ranks", fake)
    monkeypatch.setattr(bench.torch.cuda, "set_device",
                        lambda *a: pytest.fail("GPU touched before the launch"))
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7 and seen["gpus"] == 2
