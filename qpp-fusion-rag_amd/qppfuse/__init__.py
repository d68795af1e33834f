"""qppfuse — MI355X-native (gfx950) rank-fusion + QPP engine.

Drop-in for the hot path of PoisedDok/QPP-Fusion-RAG (src/fusion.py, src/qpp.py,
per-query min-max normalisation).  Host side: Python; compute: hand-written HIP
kernels in libqppfuse.so via a C-ABI (include/qppfuse.h).  See DESIGN.md.

The package re-exports the names the reference's src/__init__.py:28,37 does
(QPPBridge, compute_qpp_for_res_file, combsum, combmnz, rrf, weighted_combsum,
weighted_rrf, learned_fusion), so `from src import combsum, QPPBridge` becomes
`from qppfuse import combsum, QPPBridge`.  They resolve lazily (module
__getattr__): importing the package loads no library and touches no GPU — the
03_qpp pattern, where a parent process imports the package and forks workers
that each open their own HIP context, depends on that.
"""
from . import config as config_module
from ._lib import QPPFuseError, max_entries_per_query, version
from .config import ConfigError, config, get_qpp_index

# name -> submodule, resolved on first access (src/__init__.py:28,37)
_LAZY = {
    "QPPBridge": "qpp", "QPPResult": "qpp", "compute_qpp_for_res_file": "qpp",
    "combsum": "fusion", "combmnz": "fusion", "rrf": "fusion",
    "weighted_combsum": "fusion", "weighted_combmnz": "fusion", "weighted_rrf": "fusion",
    "learned_fusion": "fusion", "run_fusion": "fusion", "load_runs": "fusion",
    "load_qpp_scores": "fusion", "write_runfile": "fusion",
}

__all__ = ["config", "config_module", "ConfigError", "get_qpp_index", "QPPFuseError",
           "version", "max_entries_per_query"] + sorted(_LAZY)
__version__ = "0.1.0"


def __getattr__(name):
    mod = _LAZY.get(name)
    if mod is None:
        raise AttributeError(f"module 'qppfuse' has no attribute {name!r}")
    import importlib
    value = getattr(importlib.import_module(f".{mod}", __name__), name)
    globals()[name] = value  # later lookups skip this hook
    return value


def __dir__():
    return sorted(set(globals()) | set(_LAZY))
