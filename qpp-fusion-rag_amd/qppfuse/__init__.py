"""qppfuse — MI355X-native (gfx950) rank-fusion + QPP engine.

Drop-in for the hot path of PoisedDok/QPP-Fusion-RAG (src/fusion.py, src/qpp.py,
per-query min-max normalisation).  Host side: Python; compute: hand-written HIP
kernels in libqppfuse.so via a C-ABI (include/qppfuse.h).  See DESIGN.md.
"""
from . import config as config_module
from ._lib import QPPFuseError, max_entries_per_query, version
from .config import ConfigError, config, get_qpp_index

__all__ = ["config", "config_module", "ConfigError", "get_qpp_index", "QPPFuseError",
           "version", "max_entries_per_query"]
__version__ = "0.1.0"
