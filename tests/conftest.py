"""Test configuration: import paths and the `gpu` marker.

CPU tests (-m "not gpu") cover the oracle against the reference's golden
vectors, the host logic and the C-ABI surface.  GPU tests (-m gpu) are the
parity tests proper: HIP kernels through the C-ABI vs the oracle.
"""
import json
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "qpp-fusion-rag_amd"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X / gfx950)")


@pytest.fixture(scope="session")
def golden():
    return json.loads((GOLDEN / "reference_fusion.json").read_text())


@pytest.fixture(scope="session")
def golden3():
    return json.loads((GOLDEN / "reference_round3.json").read_text())


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no ROCm device is visible")
    from qppfuse import _lib
    _lib.lib()  # the HIP library must load: no fallback
    return torch.device("cuda", 0)
