"""Learned-fusion models: read the reference's pickles WITHOUT unpickling them.

The reference saves its fusion models with pickle (src/models/base.py:103-115:
{'model': <PerRetrieverLGBM | MultiOutputLGBM>, 'retrievers', 'n_qpp',
'model_type'}), and a LightGBM Booster pickles as its model text
(lightgbm.basic.Booster.__getstate__: '_handle' = model_to_string()).  This
module decodes the pickle opcode stream as DATA (dicts, lists, strings, numbers;
every class reference / constructor call becomes an inert placeholder — nothing
is imported or called), then parses the LightGBM model text into flat tree
arrays for the HIP predictor (csrc/qf_learn.hip).

Prediction semantics restated from LightGBM (>=4.0.0, requirements.txt:25; not
installed here): Booster.predict(X) uses the first best_iteration trees
(num_iteration=None -> best_iteration when > 0); a tree's output is the leaf
reached from node 0 by NumericalDecision — missing type None: fval <= threshold
goes left; Zero: |fval| <= 1e-35 takes the default side; NaN: NaN takes it, and
a NaN with another missing type is read as 0.0 — and the raw score is the
sequential double sum of the tree outputs (GBDT::PredictRaw); the regression
objective leaves it as is.
"""
from __future__ import annotations

import io
import pickletools
import re
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import numpy as np

__all__ = ["Opaque", "read_pickle_static", "Tree", "Booster", "FusionModel",
           "parse_lgbm_model", "load_fusion_model", "load_fixture", "pack_model", "PackedModel",
           "booster_texts", "model_to_fixture"]


# ------------------------------------------------------------ pickle, as data

class Opaque:
    """A pickled object reference / construction, kept inert (never resolved)."""

    def __init__(self, module: str, name: str, args: tuple = ()):
        self.module, self.name, self.args = module, name, args
        self.state: Any = None
        self.items: list = []

    def __repr__(self):
        return f"<Opaque {self.module}.{self.name}>"


_MARK = object()


def read_pickle_static(path) -> Any:
    """Decode a pickle's opcode stream into plain data; classes stay Opaque.

    Only data-building opcodes are interpreted; GLOBAL / REDUCE / NEWOBJ / BUILD /
    PERSID produce or annotate Opaque placeholders, so nothing from the file is
    ever imported or executed."""
    data = open(path, "rb").read()
    obj, _ = read_pickle_bytes(data, 0, str(path))
    return obj


def read_pickle_bytes(data: bytes, start: int = 0, what: str = "pickle") -> tuple:
    """read_pickle_static over data[start:]: (object, offset just past its STOP)."""
    stack: list = []
    memo: Dict[int, Any] = {}

    def pop_mark():
        i = len(stack) - 1
        while stack[i] is not _MARK:
            i -= 1
        items = stack[i + 1:]
        del stack[i:]
        return items

    f = io.BytesIO(data)
    f.seek(start)
    for op, arg, pos in pickletools.genops(f):  # pos: absolute offset (f.tell())
        n = op.name
        if n in ("PROTO", "FRAME"):
            continue
        if n == "STOP":
            return stack.pop(), pos + 1
        if n == "MARK":
            stack.append(_MARK)
        elif n in ("EMPTY_DICT",):
            stack.append({})
        elif n in ("EMPTY_LIST",):
            stack.append([])
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n == "EMPTY_SET":
            stack.append(set())
        elif n in ("TUPLE1", "TUPLE2", "TUPLE3"):
            k = int(n[-1])
            t = tuple(stack[-k:])
            del stack[-k:]
            stack.append(t)
        elif n == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif n == "LIST":
            stack.append(list(pop_mark()))
        elif n == "DICT":
            it = pop_mark()
            stack.append({it[i]: it[i + 1] for i in range(0, len(it), 2)})
        elif n in ("FROZENSET",):
            stack.append(frozenset(pop_mark()))
        elif n == "ADDITEMS":
            it = pop_mark()
            stack[-1].update(it)
        elif n == "APPEND":
            v = stack.pop()
            _append(stack[-1], [v])
        elif n == "APPENDS":
            it = pop_mark()
            _append(stack[-1], it)
        elif n == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            _setitems(stack[-1], [k, v])
        elif n == "SETITEMS":
            it = pop_mark()
            _setitems(stack[-1], it)
        elif n in ("MEMOIZE",):
            memo[len(memo)] = stack[-1]
        elif n in ("PUT", "BINPUT", "LONG_BINPUT"):
            memo[int(arg)] = stack[-1]
        elif n in ("GET", "BINGET", "LONG_BINGET"):
            stack.append(memo[int(arg)])
        elif n in ("SHORT_BINUNICODE", "BINUNICODE", "BINUNICODE8", "UNICODE", "STRING",
                   "BINSTRING", "SHORT_BINSTRING", "SHORT_BINBYTES", "BINBYTES", "BINBYTES8",
                   "BYTEARRAY8"):
            stack.append(arg)
        elif n in ("BININT", "BININT1", "BININT2", "LONG1", "LONG4", "INT", "LONG"):
            stack.append(arg)
        elif n in ("BINFLOAT", "FLOAT"):
            stack.append(float(arg))
        elif n == "NONE":
            stack.append(None)
        elif n == "NEWTRUE":
            stack.append(True)
        elif n == "NEWFALSE":
            stack.append(False)
        elif n == "GLOBAL":
            mod, _, name = str(arg).partition(" ")
            stack.append(Opaque(mod, name))
        elif n == "STACK_GLOBAL":
            name = stack.pop()
            mod = stack.pop()
            stack.append(Opaque(str(mod), str(name)))
        elif n in ("REDUCE", "NEWOBJ"):
            args = stack.pop()
            cls = stack.pop()
            stack.append(Opaque(getattr(cls, "module", "?"), getattr(cls, "name", "?"),
                                tuple(args) if isinstance(args, (tuple, list)) else (args,)))
        elif n == "NEWOBJ_EX":
            kwargs = stack.pop()
            args = stack.pop()
            cls = stack.pop()
            o = Opaque(getattr(cls, "module", "?"), getattr(cls, "name", "?"), tuple(args))
            o.state = {"__kwargs__": kwargs}
            stack.append(o)
        elif n == "BUILD":
            state = stack.pop()
            obj = stack[-1]
            if isinstance(obj, Opaque):
                obj.state = state
        elif n in ("PERSID", "BINPERSID"):
            pid = stack.pop() if n == "BINPERSID" else arg
            stack.append(Opaque("persistent_id", str(pid), (pid,)))
        elif n == "POP":
            stack.pop()
        elif n == "POP_MARK":
            pop_mark()
        elif n == "DUP":
            stack.append(stack[-1])
        else:
            raise ValueError(f"unsupported pickle opcode {n} in {what}")
    raise ValueError(f"{what}: pickle without STOP")


def _append(obj, items):
    if isinstance(obj, list):
        obj.extend(items)
    elif isinstance(obj, Opaque):
        obj.items.extend(items)
    else:
        raise ValueError("APPEND on a non-list")


def _setitems(obj, kv):
    if isinstance(obj, dict):
        for i in range(0, len(kv), 2):
            obj[kv[i]] = kv[i + 1]
    elif isinstance(obj, Opaque):  # e.g. defaultdict / OrderedDict subclasses
        obj.items.extend(kv)
    else:
        raise ValueError("SETITEM on a non-dict")


# --------------------------------------------------------------- LightGBM text

@dataclass
class Tree:
    num_leaves: int
    split_feature: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    threshold: np.ndarray = field(default_factory=lambda: np.zeros(0))
    decision_type: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    left_child: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    right_child: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    leaf_value: np.ndarray = field(default_factory=lambda: np.zeros(0))


@dataclass
class Booster:
    trees: List[Tree]
    best_iteration: int
    max_feature_idx: int
    objective: str

    @property
    def used_trees(self) -> List[Tree]:
        """The trees Booster.predict(X) uses: the first best_iteration (all if <= 0)."""
        n = self.best_iteration if self.best_iteration > 0 else len(self.trees)
        return self.trees[:n]


def _arr(v: str, dtype):
    return np.array([float(x) for x in v.split()], dtype=np.float64) if dtype is float else \
        np.array([int(x) for x in v.split()], dtype=dtype)


def parse_lgbm_model(text: str, best_iteration: int = 0) -> Booster:
    """LightGBM model text (v3/v4) -> Booster with numerical trees."""
    head, _, body = text.partition("\nTree=")
    hd = dict(line.split("=", 1) for line in head.splitlines() if "=" in line)
    if int(hd.get("num_tree_per_iteration", "1")) != 1 or int(hd.get("num_class", "1")) != 1:
        raise ValueError("only single-output LightGBM boosters are supported")
    objective = hd.get("objective", "regression").split()[0]
    if objective not in ("regression", "regression_l2", "l2", "mean_squared_error", "mse"):
        raise ValueError(f"LightGBM objective '{objective}' is not supported (regression only)")
    trees: List[Tree] = []
    body = "Tree=" + body
    for block in re.split(r"\n(?=Tree=)", body.split("end of trees")[0].strip()):
        kv = dict(line.split("=", 1) for line in block.strip().splitlines() if "=" in line)
        nl = int(kv["num_leaves"])
        if int(kv.get("num_cat", "0")) != 0:
            raise ValueError("categorical splits are not supported")
        if int(kv.get("is_linear", "0")) != 0:
            raise ValueError("linear trees are not supported")
        t = Tree(num_leaves=nl, leaf_value=_arr(kv["leaf_value"], float))
        if nl > 1:
            t.split_feature = _arr(kv["split_feature"], np.int32)
            t.threshold = _arr(kv["threshold"], float)
            t.decision_type = _arr(kv["decision_type"], np.int32)
            t.left_child = _arr(kv["left_child"], np.int32)
            t.right_child = _arr(kv["right_child"], np.int32)
            if np.any(t.decision_type & 1):
                raise ValueError("categorical splits are not supported")
        trees.append(t)
    return Booster(trees, int(best_iteration), int(hd.get("max_feature_idx", "-1")), objective)


@dataclass
class FusionModel:
    model_type: str
    retrievers: List[str]
    n_qpp: int
    boosters: List[Booster]  # one per retriever, in `retrievers` order


def _booster_of(obj) -> Booster:
    if not isinstance(obj, Opaque) or obj.name != "Booster" or not isinstance(obj.state, dict):
        raise ValueError("expected a pickled lightgbm Booster")
    st = obj.state
    text = st.get("_handle")
    if isinstance(text, bytes):
        text = text.decode()
    if not isinstance(text, str) or not text.startswith("tree"):
        raise ValueError("Booster without model text")
    return parse_lgbm_model(text, int(st.get("best_iteration", 0) or 0))


def model_to_fixture(model: FusionModel, texts: List[str]) -> dict:
    return {"model_type": model.model_type, "retrievers": model.retrievers,
            "n_qpp": model.n_qpp,
            "boosters": [{"best_iteration": b.best_iteration, "text": t}
                         for b, t in zip(model.boosters, texts)]}


def booster_texts(path) -> List[str]:
    """The model text of every booster of a fusion pickle, in booster order."""
    top = read_pickle_static(path)
    st = top["model"].state
    models = st["models"]
    objs = models if isinstance(models, list) else [models[r] for r in st["retrievers"]]
    return [o.state["_handle"] if isinstance(o.state["_handle"], str)
            else o.state["_handle"].decode() for o in objs]


def load_fixture(path) -> FusionModel:
    """A model saved as JSON (tests/golden/lgbm/*.json.gz): the same content as the
    pickle — model type, retrievers, n_qpp, and each booster's text + best_iteration."""
    import gzip
    import json
    opener = gzip.open if str(path).endswith(".gz") else open
    with opener(path, "rt") as fh:
        d = json.load(fh)
    return FusionModel(d["model_type"], list(d["retrievers"]), int(d["n_qpp"]),
                       [parse_lgbm_model(b["text"], int(b["best_iteration"]))
                        for b in d["boosters"]])


def load_fusion_model(path) -> FusionModel:
    """The reference's learned-fusion pickle (src/fusion.py:407-413) -> FusionModel.

    `.json` / `.json.gz` paths are read as fixtures (load_fixture)."""
    if str(path).endswith((".json", ".json.gz")):
        return load_fixture(path)
    top = read_pickle_static(path)
    if not isinstance(top, dict) or "model" not in top:
        raise ValueError(f"{path}: not a fusion model pickle")
    model = top["model"]
    model_type = top.get("model_type", "PerRetrieverLGBM")
    st = model.state if isinstance(model, Opaque) and isinstance(model.state, dict) else {}
    retrievers = list(top.get("retrievers") or st.get("retrievers") or [])
    n_qpp = int(top.get("n_qpp", st.get("n_qpp", 13)))
    models = st.get("models")
    if model_type == "MultiOutputLGBM" and isinstance(models, list):
        boosters = [_booster_of(b) for b in models]
    elif model_type == "PerRetrieverLGBM" and isinstance(models, dict):
        boosters = [_booster_of(models[r]) for r in retrievers]
    else:
        raise NotImplementedError(
            f"learned fusion model '{model_type}' is not a LightGBM model (MultiOutputLGBM / "
            f"PerRetrieverLGBM; FusionMLP pickles load through qppfuse.mlp.load_mlp_model)")
    if len(boosters) != len(retrievers):
        raise ValueError("model has a different number of boosters and retrievers")
    return FusionModel(model_type, retrievers, n_qpp, boosters)


# ------------------------------------------------------------- device packing

@dataclass
class PackedModel:
    """Flat arrays for qf_gbdt_predict (include/qppfuse.h)."""
    n_boosters: int
    n_features: int
    tree_off: np.ndarray    # int32 [B+1]: trees of booster b
    node_off: np.ndarray    # int32 [T+1]: internal nodes of tree t
    leaf_off: np.ndarray    # int32 [T+1]: leaves of tree t
    feature: np.ndarray     # int32 [nodes]
    threshold: np.ndarray   # float64 [nodes]
    dtype: np.ndarray       # int32 [nodes] LightGBM decision_type
    left: np.ndarray        # int32 [nodes] child: >= 0 node, < 0 leaf ~index
    right: np.ndarray       # int32 [nodes]
    leaf_value: np.ndarray  # float64 [leaves]
    _dev: dict = field(default_factory=dict, repr=False)

    def to_device(self, device):
        """Device copies (cached): the arrays qf_gbdt_predict reads."""
        import torch
        if not self._dev:
            for k in ("tree_off", "node_off", "leaf_off", "feature", "threshold", "dtype",
                      "left", "right", "leaf_value"):
                a = getattr(self, k)
                if a.size == 0:  # a model of single-leaf trees has no nodes
                    a = np.zeros(1, a.dtype)
                self._dev[k] = torch.from_numpy(np.ascontiguousarray(a)).to(device)
        return self._dev


def pack_model(model: FusionModel) -> PackedModel:
    tree_off, node_off, leaf_off = [0], [0], [0]
    feat, thr, dt, lc, rc, lv = [], [], [], [], [], []
    nf = model.n_qpp * len(model.retrievers)
    for b in model.boosters:
        for t in b.used_trees:
            if t.num_leaves > 1:
                if int(t.split_feature.max()) >= nf:
                    raise ValueError("a split uses a feature beyond n_qpp * n_retrievers")
                feat.append(t.split_feature)
                thr.append(t.threshold)
                dt.append(t.decision_type)
                lc.append(t.left_child)
                rc.append(t.right_child)
            node_off.append(node_off[-1] + max(t.num_leaves - 1, 0))
            lv.append(t.leaf_value[: t.num_leaves])
            leaf_off.append(leaf_off[-1] + t.num_leaves)
        tree_off.append(len(node_off) - 1)
    cat = lambda xs, d: np.concatenate(xs).astype(d) if xs else np.zeros(0, d)
    return PackedModel(len(model.boosters), nf, np.asarray(tree_off, np.int32),
                       np.asarray(node_off, np.int32), np.asarray(leaf_off, np.int32),
                       cat(feat, np.int32), cat(thr, np.float64), cat(dt, np.int32),
                       cat(lc, np.int32), cat(rc, np.int32), cat(lv, np.float64))
