"""The configuration keys the fusion/QPP path reads, loaded like the reference loads them.

The reference's Config singleton (src/config.py:100-193) reads
config/defaults.yaml with yaml.safe_load and expands ${VAR} / ${VAR:default}
in every string value (ENV_PATTERN, src/config.py:115,159-193).  This module
does the same for the keys on this path:

  qpp.n_methods / methods / method_index / default_method / default_index /
  normalization                       config/defaults.yaml:159-200
  fusion.rrf_k / methods              config/defaults.yaml:205-217
  processing.retrieval.top_k / first_stage_k   config/defaults.yaml:152-154
  evaluation.ir_metrics               config/defaults.yaml:224-234

The YAML is found, in order, at $QPPFUSE_CONFIG, at
$PROJECT_ROOT/config/defaults.yaml (the reference's own location, src/config.py:
130-136), or at ./config/defaults.yaml; without one the built-in values below
(the reference's shipped defaults) are used.  A key the YAML does not set keeps
its built-in value.  Environment plumbing for retrievers / LLMs
(src/config.py:195-231: cache dirs, thread counts, Java options) is out of scope.

`config` is one object for the life of the process (modules hold it by
reference, as the reference's modules hold its singleton); load_config()
refreshes it in place.
"""
from __future__ import annotations

import copy
import os
import re
from pathlib import Path
from typing import Any, Dict, Optional


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

DEFAULTS: Dict[str, Any] = {
    "qpp": {"n_methods": 13, "methods": list(QPP_METHODS),
            "method_index": dict(QPP_METHOD_INDEX), "default_method": "RSD",
            "default_index": 5, "normalization": "minmax"},
    "fusion": {"rrf_k": 60, "methods": list(FUSION_METHODS)},
    "processing": {"retrieval": {"top_k": 100, "first_stage_k": 100}},
    "evaluation": {"ir_metrics": ["nDCG@5", "nDCG@10", "nDCG@20", "RR@5", "RR@10", "R@5",
                                  "R@10", "R@100", "P@10", "AP"]},
}
_SECTIONS = {"qpp": None, "fusion": None, "processing": ("retrieval",), "evaluation": None}

# ${VAR} or ${VAR:default} (src/config.py:115)
ENV_PATTERN = re.compile(r'\$\{([^}:]+)(?::([^}]*))?\}')


def _expand_string(s: str) -> str:
    def repl(m):
        val = os.environ.get(m.group(1))
        if val is not None:
            return val
        if m.group(2) is not None:
            return m.group(2)
        raise ConfigError(f"Environment variable '{m.group(1)}' not set and no default provided.\n"
                          f"Set it or provide default in config: ${{{m.group(1)}:default_value}}")
    return ENV_PATTERN.sub(repl, s)


def expand_env_vars(obj: Any) -> Any:
    """Recursive ${VAR[:default]} expansion of string values (src/config.py:159-174)."""
    if isinstance(obj, dict):
        return {k: expand_env_vars(v) for k, v in obj.items()}
    if isinstance(obj, list):
        return [expand_env_vars(v) for v in obj]
    if isinstance(obj, str):
        return _expand_string(obj)
    return obj


class Section:
    """Attribute and item access over one mapping (the reference's ConfigDict)."""

    def __init__(self, data: Dict[str, Any]):
        object.__setattr__(self, "_data", {})
        self._set(data)

    def _set(self, data: Dict[str, Any]) -> None:
        self._data.clear()
        for k, v in data.items():
            self._data[k] = Section(v) if isinstance(v, dict) and k != "method_index" else v

    def __getattr__(self, key):
        try:
            return self._data[key]
        except KeyError:
            raise AttributeError(f"Config has no key '{key}'") from None

    def __setattr__(self, key, value):
        self._data[key] = value

    def __getitem__(self, key):
        return self._data[key]

    def __contains__(self, key):
        return key in self._data

    def get(self, key, default=None):
        return self._data.get(key, default)

    def to_dict(self) -> Dict[str, Any]:
        return {k: v.to_dict() if isinstance(v, Section) else copy.deepcopy(v)
                for k, v in self._data.items()}

    def __repr__(self):
        return f"Section({self.to_dict()})"


def _merge(base: Dict[str, Any], over: Dict[str, Any]) -> Dict[str, Any]:
    out = copy.deepcopy(base)
    for k, v in (over or {}).items():
        if k in out and isinstance(out[k], dict) and isinstance(v, dict) and k != "method_index":
            out[k] = _merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def find_config_file() -> Optional[Path]:
    """QPPFUSE_CONFIG, else <PROJECT_ROOT>/config/defaults.yaml (the reference reads
    <project_root>/config/defaults.yaml only, src/config.py:100-146) — never a file
    that merely happens to sit in the working directory."""
    cands = []
    if os.environ.get("QPPFUSE_CONFIG"):
        cands.append(Path(os.environ["QPPFUSE_CONFIG"]))
    if os.environ.get("PROJECT_ROOT"):
        cands.append(Path(os.environ["PROJECT_ROOT"]) / "config" / "defaults.yaml")
    for c in cands:
        if c.is_file():
            return c
    return None


class Config(Section):
    """The path's slice of the reference's Config singleton."""

    def __init__(self):
        super().__init__({})
        object.__setattr__(self, "source", None)
        self.load()

    def load(self, path: Optional[os.PathLike] = None) -> "Config":
        """(Re)load from `path`, else from find_config_file(), else the built-in values."""
        p = Path(path) if path is not None else find_config_file()
        if p is not None and not p.is_file():
            raise ConfigError(f"Configuration file not found: {p}")
        raw = {}
        if p is not None:
            import yaml  # only when a file is actually read
            with open(p, "r") as fh:
                raw = yaml.safe_load(fh) or {}
        raw = expand_env_vars({k: raw[k] for k in _SECTIONS if k in raw})
        merged = _merge(DEFAULTS, raw)
        self._set(merged)
        object.__setattr__(self, "source", str(p) if p is not None else None)
        return self

    def get_qpp_index(self, method_name: str) -> int:
        return get_qpp_index(method_name)


config = Config()


def load_config(path: Optional[os.PathLike] = None) -> Config:
    """Reload the process-wide `config` in place (every module sees the new values)."""
    return config.load(path)


def get_qpp_index(method_name: str) -> int:
    """Case-insensitive QPP name -> column; "fusion" -> -1 (src/config.py:317-333)."""
    method_index = config.qpp.method_index
    for name, idx in method_index.items():
        if name.lower() == method_name.lower():
            return idx
    if method_name.lower() == "fusion":
        return -1
    raise ConfigError(f"Unknown QPP method: {method_name}. "
                      f"Valid: {list(method_index.keys())} or 'fusion'")
