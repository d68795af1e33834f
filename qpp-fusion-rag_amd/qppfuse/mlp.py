"""FusionMLP learned-fusion models, read statically, for qf_mlp_weights.

The reference saves FusionMLP (src/models/mlp_model.py:276-301) with plain
pickle: {'model': the FusionMLP object (its nn.Sequential inside), 'model_state':
state_dict, 'retrievers', 'n_qpp', 'hidden_sizes', 'dropout', 'model_type':
'FusionMLP', 'is_trained'}.  learned_fusion (src/fusion.py:407-429) unpickles it
and calls model.predict(X), so the weights that count are the object's own
Sequential.  Tensors in a plain pickle are
`torch._utils._rebuild_tensor_v2(storage, offset, size, stride, ...)` whose
storage is `torch.storage._load_from_bytes(blob)`, a legacy torch.save stream:
five pickles (magic number, protocol version, system info, the storage as a
persistent id ('storage', <type>, key, location, numel), the key list) and
then, per key, an int64 element count and the raw little-endian elements.
All of it is decoded here as data (qppfuse.lgbm.read_pickle_bytes): nothing
from the file is imported or executed.

What predict computes (src/models/mlp_model.py:254-274): _filter_features
(X[:, j*n_qpp + qpp_indices[k]] -> column j*n_used + k, only when fewer than
n_qpp indices are used), torch.FloatTensor, Linear -> ReLU -> Dropout (identity
in eval) ... -> Linear, softmax, then _normalize_weights (src/models/
base.py:120-125).  The device does it in qf_mlp_weights (csrc/qf_learn.hip).
"""
from __future__ import annotations

import base64
import gzip
import json
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from .lgbm import Opaque, read_pickle_bytes, read_pickle_static

__all__ = ["MLPModel", "decode_storage", "decode_tensor", "load_mlp_model", "load_mlp_fixture",
           "mlp_to_fixture", "is_mlp_pickle"]

_STORAGE_DTYPES = {"FloatStorage": np.float32, "DoubleStorage": np.float64,
                   "HalfStorage": np.float16, "LongStorage": np.int64, "IntStorage": np.int32}


@dataclass
class MLPModel:
    """A FusionMLP's inference content: layers [(W [out, in] f32, b [out] f32)]."""
    retrievers: List[str]
    n_qpp: int
    qpp_indices: List[int]
    layers: list
    model_type: str = "FusionMLP"
    _dev: dict = field(default_factory=dict, repr=False)

    @property
    def n_outputs(self) -> int:
        return int(self.layers[-1][0].shape[0])

    def input_columns(self) -> np.ndarray:
        """Column of learned_fusion's X feeding each model input (_filter_features,
        src/models/mlp_model.py:104-122; X as is when all n_qpp are used)."""
        R, n_used = len(self.retrievers), len(self.qpp_indices)
        if n_used >= self.n_qpp:
            return np.arange(R * self.n_qpp, dtype=np.int32)
        return np.asarray([j * self.n_qpp + i for j in range(R) for i in self.qpp_indices],
                          np.int32)

    def widths(self) -> List[int]:
        return [int(self.layers[0][0].shape[1])] + [int(W.shape[0]) for W, _ in self.layers]

    def flat_params(self) -> np.ndarray:
        return np.concatenate([np.concatenate([W.reshape(-1), b.reshape(-1)])
                               for W, b in self.layers]).astype(np.float32)

    def to_device(self, device):
        """(in_col int32, params float32) on the device, cached."""
        import torch
        if not self._dev:
            self._dev["in_col"] = torch.from_numpy(self.input_columns()).to(device)
            self._dev["params"] = torch.from_numpy(self.flat_params()).to(device)
        return self._dev

    def validate(self) -> None:
        w = self.widths()
        if len(self.input_columns()) != w[0]:
            raise ValueError(f"the model takes {w[0]} inputs but its QPP selection gives "
                             f"{len(self.input_columns())}")
        for (W, b), n_in, n_out in zip(self.layers, w[:-1], w[1:]):
            if W.shape != (n_out, n_in) or b.shape != (n_out,):
                raise ValueError("inconsistent Linear layer shapes")
        if w[-1] != len(self.retrievers):
            raise ValueError(f"the model predicts {w[-1]} weights for "
                             f"{len(self.retrievers)} retrievers")


def decode_storage(blob: bytes) -> np.ndarray:
    """torch.storage._load_from_bytes(blob) as data: the legacy torch.save stream of
    one storage -> its elements (1-D numpy array)."""
    pos = 0
    for _ in range(3):  # magic number, protocol version, system info
        _, pos = read_pickle_bytes(blob, pos, "storage")
    obj, pos = read_pickle_bytes(blob, pos, "storage")
    keys, pos = read_pickle_bytes(blob, pos, "storage")
    if not (isinstance(obj, Opaque) and obj.module == "persistent_id" and obj.args
            and isinstance(obj.args[0], tuple) and obj.args[0][0] == "storage"):
        raise ValueError("not a legacy torch storage stream")
    pid = obj.args[0]
    stype = pid[1].name if isinstance(pid[1], Opaque) else str(pid[1])
    if stype not in _STORAGE_DTYPES:
        raise NotImplementedError(f"storage type {stype}")
    if list(keys) != [pid[2]]:
        raise ValueError("a storage stream holding other storages")
    dt = np.dtype(_STORAGE_DTYPES[stype]).newbyteorder("<")
    n = int(np.frombuffer(blob, "<i8", 1, pos)[0])
    data = np.frombuffer(blob, dt, n, pos + 8)
    if n != int(pid[4]):
        raise ValueError("storage element count mismatch")
    return data.astype(dt.newbyteorder("="))


def decode_tensor(t) -> np.ndarray:
    """_rebuild_parameter / _rebuild_tensor_v2(storage, offset, size, stride, ...)."""
    if isinstance(t, Opaque) and t.name == "_rebuild_parameter":
        t = t.args[0]
    if not (isinstance(t, Opaque) and t.name == "_rebuild_tensor_v2"):
        raise ValueError(f"not a tensor: {t!r}")
    st, offset, size, stride = t.args[0], int(t.args[1]), tuple(t.args[2]), tuple(t.args[3])
    if not (isinstance(st, Opaque) and st.name == "_load_from_bytes"):
        raise NotImplementedError("tensor storage is not an inline byte stream")
    flat = decode_storage(st.args[0])
    # the geometry comes from the file: check it lies inside the storage before
    # as_strided (which would read out of bounds on a corrupt or hostile pickle)
    if len(size) != len(stride):
        raise ValueError("tensor size / stride rank mismatch")
    if offset < 0 or offset > len(flat) or any(s < 0 for s in size) or any(s < 0 for s in stride):
        raise ValueError("tensor offset / size / stride out of range")
    if all(s > 0 for s in size) and offset + sum((s - 1) * st_ for s, st_ in zip(size, stride)) >= len(flat):
        raise ValueError("tensor view extends past its storage")
    it = flat.itemsize
    view = np.lib.stride_tricks.as_strided(flat[offset:], shape=size,
                                           strides=tuple(s * it for s in stride))
    return np.array(view)


def _sequential_layers(seq) -> list:
    """nn.Sequential of Linear / ReLU / Dropout -> [(W, b)] (ReLU between Linear
    layers, as FusionMLP._build_model lays them out, src/models/mlp_model.py:86-102)."""
    if not (isinstance(seq, Opaque) and seq.name == "Sequential" and isinstance(seq.state, dict)):
        raise NotImplementedError("FusionMLP without an nn.Sequential")
    mods = seq.state["_modules"]
    items = list(mods.items()) if isinstance(mods, dict) else \
        [(mods.items[i], mods.items[i + 1]) for i in range(0, len(mods.items), 2)]
    layers, pattern = [], []
    for _, mod in items:
        name = mod.name if isinstance(mod, Opaque) else repr(mod)
        if name == "Linear":
            prm = mod.state["_parameters"]
            prm = prm if isinstance(prm, dict) else \
                {prm.items[i]: prm.items[i + 1] for i in range(0, len(prm.items), 2)}
            W = decode_tensor(prm["weight"]).astype(np.float32)
            b = decode_tensor(prm["bias"]).astype(np.float32) if prm.get("bias") is not None \
                else np.zeros(W.shape[0], np.float32)
            layers.append((W, b))
            pattern.append("L")
        elif name == "ReLU":
            pattern.append("R")
        elif name == "Dropout":
            continue  # identity in eval mode
        else:
            raise NotImplementedError(f"FusionMLP layer {name} is not supported on device")
    if "".join(pattern) != "LR" * (len(layers) - 1) + "L":
        raise NotImplementedError(f"FusionMLP layout {''.join(pattern)} (expected (Linear ReLU)* "
                                  f"Linear)")
    return layers


def is_mlp_pickle(top) -> bool:
    return isinstance(top, dict) and top.get("model_type") == "FusionMLP"


def mlp_from_pickle_dict(top) -> MLPModel:
    obj = top["model"]
    st = obj.state if isinstance(obj, Opaque) and isinstance(obj.state, dict) else {}
    retrievers = list(st.get("retrievers") or top.get("retrievers") or [])
    n_qpp = int(st.get("n_qpp", top.get("n_qpp", 13)))
    qpp_indices = [int(i) for i in st.get("qpp_indices", [5])]
    m = MLPModel(retrievers, n_qpp, qpp_indices, _sequential_layers(st.get("model")))
    m.validate()
    return m


def load_mlp_model(path) -> MLPModel:
    """The reference's fusion_mlp.pkl (or a fixture .json[.gz]) -> MLPModel."""
    if str(path).endswith((".json", ".json.gz")):
        return load_mlp_fixture(path)
    top = read_pickle_static(path)
    if not is_mlp_pickle(top):
        raise ValueError(f"{path}: not a FusionMLP pickle")
    return mlp_from_pickle_dict(top)


def _b64(a: np.ndarray) -> str:
    return base64.b64encode(np.ascontiguousarray(a, "<f4").tobytes()).decode()


def mlp_to_fixture(m: MLPModel) -> dict:
    return {"model_type": "FusionMLP", "retrievers": m.retrievers, "n_qpp": m.n_qpp,
            "qpp_indices": m.qpp_indices,
            "layers": [{"out": int(W.shape[0]), "in": int(W.shape[1]), "W": _b64(W),
                        "b": _b64(b)} for W, b in m.layers]}


def load_mlp_fixture(path) -> MLPModel:
    opener = gzip.open if str(path).endswith(".gz") else open
    with opener(path, "rt") as fh:
        d = json.load(fh)
    layers = []
    for L in d["layers"]:
        W = np.frombuffer(base64.b64decode(L["W"]), "<f4").reshape(L["out"], L["in"])
        b = np.frombuffer(base64.b64decode(L["b"]), "<f4")
        layers.append((W.astype(np.float32), b.astype(np.float32)))
    m = MLPModel(list(d["retrievers"]), int(d["n_qpp"]), [int(i) for i in d["qpp_indices"]],
                 layers)
    m.validate()
    return m


def model_kind(path) -> Optional[str]:
    """'FusionMLP' for an MLP pickle / fixture, else None (LightGBM)."""
    p = str(path)
    if p.endswith((".json", ".json.gz")):
        opener = gzip.open if p.endswith(".gz") else open
        with opener(p, "rt") as fh:
            return "FusionMLP" if json.load(fh).get("model_type") == "FusionMLP" else None
    top = read_pickle_static(p)
    return "FusionMLP" if is_mlp_pickle(top) else None
