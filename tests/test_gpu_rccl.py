"""The RCCL (backend "nccl") form of the path's collectives on a real device.

The 8-GPU run is the driver's; a one-GPU box can still run the nccl backend at
world size 1 under torch.distributed.run, which exercises the same process-group
init (device_id bound), the MIN all-reduce of the QPP [min, -max] buffer and the
async fused top-k gather on device buffers that bench.py times at N > 1.  The
N > 1 arithmetic is covered by the gloo world-2 tests (tests/test_dist.py).
"""
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.gpu
def test_rccl_collectives_world1(gpu):
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={port}",
           str(ROOT / "tests" / "rccl_rank.py")]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "rccl-ok" in r.stdout
