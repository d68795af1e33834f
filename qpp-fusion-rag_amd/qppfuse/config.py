"""The configuration keys the fusion/QPP path reads.

Mirrors the values of the reference's config/defaults.yaml that this path uses
(qpp.* :159-200, fusion.* :205-217, processing.retrieval.top_k :152-154,
evaluation.ir_metrics :224-234) and
Config.get_qpp_index (src/config.py:317-333).  Environment plumbing for
retrievers / LLMs (src/config.py:195-231) is out of scope.
"""
from __future__ import annotations

from types import SimpleNamespace


class ConfigError(Exception):
    """Unknown configuration key or value (src/config.py ConfigError)."""


# Java output order, config/defaults.yaml:164-177 (also the .qpp column order).
QPP_METHODS = ["nqc", "smv", "wig", "SigmaMax", "SigmaX", "RSD", "UEF", "MaxIDF", "avgidf",
               "cumnqc", "snqc", "dense-qpp", "dense-qpp-m"]
# Name -> column index used for weighting, config/defaults.yaml:180-193.  NOTE: the
# names do not match the Java column at that index; this
# table is reproduced verbatim so weights select the same column as the reference.
QPP_METHOD_INDEX = {"SMV": 0, "Sigma_max": 1, "Sigma(%)": 2, "NQC": 3, "UEF": 4, "RSD": 5,
                    "QPP-PRP": 6, "WIG": 7, "SCNQC": 8, "QV-NQC": 9, "DM": 10, "NQA-QPP": 11,
                    "BERTQPP": 12}
FUSION_METHODS = ["combsum", "combmnz", "rrf", "wcombsum", "wcombmnz", "wrrf", "learned"]

config = SimpleNamespace(
    qpp=SimpleNamespace(n_methods=13, methods=list(QPP_METHODS),
                        method_index=dict(QPP_METHOD_INDEX), default_method="RSD",
                        default_index=5, normalization="minmax"),
    fusion=SimpleNamespace(rrf_k=60, methods=list(FUSION_METHODS)),
    processing=SimpleNamespace(retrieval=SimpleNamespace(top_k=100, first_stage_k=100)),
    # config/defaults.yaml:224-234 (evaluation.ir_metrics)
    evaluation=SimpleNamespace(ir_metrics=["nDCG@5", "nDCG@10", "nDCG@20", "RR@5", "RR@10",
                                           "R@5", "R@10", "R@100", "P@10", "AP"]),
)


def get_qpp_index(method_name: str) -> int:
    """Case-insensitive QPP name -> column; "fusion" -> -1 (src/config.py:317-333)."""
    for name, idx in config.qpp.method_index.items():
        if name.lower() == method_name.lower():
            return idx
    if method_name.lower() == "fusion":
        return -1
    raise ConfigError(f"Unknown QPP method: {method_name}. "
                      f"Valid: {list(config.qpp.method_index.keys())} or 'fusion'")


config.get_qpp_index = get_qpp_index
