"""Faithful Python port of the reference hot path — TEST INFRASTRUCTURE ONLY.

Restates, algorithm for algorithm, what PoisedDok/QPP-Fusion-RAG runs on the
CPU, so that (a) small parity cases have a pure-Python checker independent of
the C oracle and the GPU kernels, and (b) bench.py's cpu_baseline times the
reference's own per-row algorithm ("port") on the GPU box's host cores.

 - weighted fusions: pandas groupby + per-row iterrows loop
   (src/fusion.py:237-380), first-seen output order;
 - unweighted fusions: the reference converts DataFrames to ranx Runs with an
   iterrows loop (src/fusion.py:455-466) and calls ranx.fuse (not installed:
   restated from ranx's published semantics — min-max per run & query, comb
   sum / mnz, reciprocal rank on the score-sorted run), then sorts
   (src/fusion.py:469-477);
 - write_runfile (src/fusion.py:480-492), normalize_scores
   (src/retrievers/base.py:60-73), _normalize_qpp (src/qpp.py:340-374);
 - QPPBridge.computeQPPScores restated in Python (QPPBridge.java:134-453).

Never imported by the product.
"""
from __future__ import annotations

import math
from collections import defaultdict
from typing import Dict, List, Tuple

import pandas as pd

Fused = Dict[str, List[Tuple[str, float]]]


# ---------------------------------------------------------------- fusion ----

def qpp_weight(qid, ranker, qpp_data, qpp_index, fusion_mode):
    """get_qpp_weight semantics (src/fusion.py:116-158)."""
    if qid not in qpp_data:
        raise KeyError(f"QPP data missing for query '{qid}'. Run QPP computation first.")
    if ranker not in qpp_data[qid]:
        raise KeyError(f"QPP data missing for ranker '{ranker}' on query '{qid}'. "
                       f"Available: {list(qpp_data[qid].keys())}")
    vals = qpp_data[qid][ranker]
    if fusion_mode or qpp_index == -1:
        return sum(vals) / len(vals)
    if qpp_index >= len(vals):
        raise IndexError(f"QPP index {qpp_index} out of range. Available: 0-{len(vals)-1}")
    return vals[qpp_index]


def weighted_fusion(runs: Dict[str, pd.DataFrame], qpp_data, qpp_index: int, kind: str,
                    k: int = 60) -> Fused:
    """kind in {"wcombsum", "wcombmnz", "wrrf"}; the reference's per-row loop."""
    qids = sorted(set().union(*[set(df["qid"].unique()) for df in runs.values()]))
    fusion_mode = qpp_index == -1
    by_ranker = {name: df.groupby("qid") for name, df in runs.items()}
    out: Fused = {}
    for qid in qids:
        acc = defaultdict(float)
        count = defaultdict(int)
        for name, groups in by_ranker.items():
            w = qpp_weight(qid, name, qpp_data, qpp_index, fusion_mode)
            if qid not in groups.groups:
                continue
            rows = groups.get_group(qid)
            if kind == "wrrf":
                rows = rows.sort_values("rank")
            for _, row in rows.iterrows():
                if kind == "wrrf":
                    acc[row["docno"]] += w / (k + row["rank"])
                else:
                    acc[row["docno"]] += w * row["score"]
                    count[row["docno"]] += 1
        if kind == "wcombmnz":
            out[qid] = [(d, s * count[d]) for d, s in acc.items()]
        else:
            out[qid] = list(acc.items())
    return out


def _to_run_dicts(runs: Dict[str, pd.DataFrame]):
    """_df_runs_to_ranx: {name: {qid: {docno: score}}} via iterrows (later rows win)."""
    res = {}
    for name, df in runs.items():
        rd: Dict[str, Dict[str, float]] = {}
        for _, row in df.iterrows():
            rd.setdefault(str(row["qid"]), {})[str(row["docno"])] = float(row["score"])
        res[name] = rd
    return res


def _minmax(d: Dict[str, float]) -> Dict[str, float]:
    if not d:
        return {}
    lo, hi = min(d.values()), max(d.values())
    den = max(hi - lo, 1e-9)  # ranx min_max_norm's denominator ("avoid division by zero")
    return {doc: ((s - lo) / den if den > 0 else 0.0) for doc, s in d.items()}


def ranx_fusion(runs: Dict[str, pd.DataFrame], kind: str, k: int = 60) -> Fused:
    """kind in {"combsum", "combmnz", "rrf"} with ranx semantics."""
    run_dicts = list(_to_run_dicts(runs).values())
    qids = sorted(set().union(*[set(r.keys()) for r in run_dicts]))
    out: Fused = {}
    for qid in qids:
        acc: Dict[str, float] = {}
        cnt: Dict[str, int] = {}
        for rd in run_dicts:
            norm = _minmax(rd.get(qid, {}))
            if kind == "rrf":
                ranked = sorted(norm.items(), key=lambda x: -x[1])
                contrib = [(doc, 1.0 / (k + i + 1)) for i, (doc, _) in enumerate(ranked)]
            else:
                contrib = list(norm.items())
            for doc, c in contrib:
                acc[doc] = acc.get(doc, 0.0) + c
                cnt[doc] = cnt.get(doc, 0) + 1
        if kind == "combmnz":
            acc = {doc: s * cnt[doc] for doc, s in acc.items()}
        out[qid] = sorted(acc.items(), key=lambda x: -x[1])
    return out


def fuse(runs, method: str, qpp_data=None, qpp_index: int = 5, k: int = 60) -> Fused:
    if method in ("combsum", "combmnz", "rrf"):
        return ranx_fusion(runs, method, k)
    return weighted_fusion(runs, qpp_data, qpp_index, method, k)


def qid_sort_key(x: str):
    return int(x.replace("test", "")) if x.startswith("test") else x


def runfile_text(fused: Fused, tag: str) -> str:
    """Bytes write_runfile would produce (src/fusion.py:480-492)."""
    out = []
    for qid in sorted(fused.keys(), key=qid_sort_key):
        ranked = sorted(fused[qid], key=lambda x: x[1], reverse=True)
        for rank, (doc, score) in enumerate(ranked, start=1):
            out.append(f"{qid} Q0 {doc} {rank} {score:.6f} {tag}\n")
    return "".join(out)


def normalize_scores(results):
    """BaseRetriever.normalize_scores (src/retrievers/base.py:60-73)."""
    if not results:
        return []
    vals = [s for _, s, _ in results]
    lo, hi = min(vals), max(vals)
    rng = hi - lo if hi > lo else 1.0
    return [(doc, (s - lo) / rng, r) for doc, s, r in results]


# ------------------------------------------------------------------- QPP ----

def _jdk_average(vals, default):
    """DoubleStream.average(): compensated sum (JDK 11-17 computeFinalSum)."""
    if not vals:
        return default
    s = c = simple = 0.0
    for v in vals:
        tmp = v - c
        velvel = s + tmp
        c = (velvel - s) - tmp
        s = velvel
        simple += v
    tot = s + c
    if math.isnan(tot) and math.isinf(simple):
        tot = simple
    return tot / len(vals)


def _f32(x: float) -> float:
    """Gson's getAsFloat of the JSON number json.dumps wrote (QPPBridge.java:67-70,
    src/qpp.py:130-147): Float.parseFloat(repr(x)), a correctly rounded
    decimal -> float conversion — glibc's strtof is one (ISO C / IEEE 754)."""
    import ctypes
    global _STRTOF
    if _STRTOF is None:
        _STRTOF = ctypes.CDLL(None).strtof
        _STRTOF.restype = ctypes.c_float
        _STRTOF.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
    return float(_STRTOF(repr(float(x)).encode(), None))


_STRTOF = None


def java_qpp(num_terms_raw: int, maxidf: float, avgidf: float, scores) -> Dict[str, float]:
    """computeQPPScores for one list (QPPBridge.java:134-191); {} for no scores."""
    if len(scores) == 0:
        return {}
    r = [_f32(float(s)) for s in scores][:50]
    n = len(r)
    nt = max(1, num_terms_raw)

    def nqc(a):
        if not a:
            return 0.0
        m = _jdk_average(a, 0.0)
        acc = 0.0
        for v in a:
            acc += (v - m) * (v - m)
        return acc / len(a)

    mean = _jdk_average(r, 0.0)
    out = {}
    out["nqc"] = nqc(r)
    mu_hat = _jdk_average(r, 1.0)
    mu_hat = 1.0 if mu_hat <= 0 else mu_hat
    smv = 0.0
    for v in r:
        if v > 0:
            smv += v * abs(math.log(v / mu_hat))
    out["smv"] = smv / n
    base = 1.0 / max(0.01, _jdk_average(r, 1.0))
    wig = 0.0
    for v in r:
        wig += v - base
    out["wig"] = wig / (nt * n)
    if n < 2:
        out["SigmaMax"] = 0.0
    else:
        best = 0.0
        for m in range(2, n + 1):
            pm = _jdk_average(r[:m], 0.0)
            var = _jdk_average([(v - pm) * (v - pm) for v in r[:m]], 0.0)
            best = max(best, math.sqrt(var))
        out["SigmaMax"] = best / math.sqrt(max(1, nt))
    sx = 0.0
    if n >= 2:
        thr = r[0] * 0.5
        f = [v for v in r if v >= thr]
        if len(f) >= 2:
            fm = _jdk_average(f, 0.0)
            sx = math.sqrt(_jdk_average([(v - fm) * (v - fm) for v in f], 0.0))
    out["SigmaX"] = sx
    rsd = 0.0
    if n >= 3:
        sd = math.sqrt(_jdk_average([(v - mean) * (v - mean) for v in r], 0.0))
        if sd >= 1e-10:
            sk = 0.0
            for v in r:
                sk += math.pow((v - mean) / sd, 3)
            rsd = sk / n
    out["RSD"] = rsd
    util = wsum = 0.0
    for i in range(min(20, n)):
        w = 1.0 / (math.log(i + 2) / math.log(2))
        util += r[i] * w
        wsum += w
    out["UEF"] = util / wsum
    out["MaxIDF"] = maxidf
    out["avgidf"] = avgidf
    if n < 2:
        out["cumnqc"] = 0.0
    else:
        cum = 0.0
        for m in range(2, n + 1):
            cum += nqc(r[:m])
        out["cumnqc"] = cum / (n - 1)
    if mean <= 0:
        out["snqc"] = 0.0
    else:
        acc = 0.0
        for v in r:
            if v <= 0:
                continue
            f2 = (v - mean) * (v - mean) / v
            prod = math.pow(1.0, 0.33) * math.pow(f2, 0.33)
            acc += math.pow(prod, 0.33)
        out["snqc"] = acc / n
    if n < 2:
        spread = 0.0
    else:
        rng = max(r) - min(r)
        spread = math.log(1 + 1.0 / rng) if rng > 0 else 0.0
    out["dense-qpp"] = spread
    out["dense-qpp-m"] = spread
    return out


QPP_NAMES = ["nqc", "smv", "wig", "SigmaMax", "SigmaX", "RSD", "UEF", "MaxIDF", "avgidf",
             "cumnqc", "snqc", "dense-qpp", "dense-qpp-m"]


def normalize_qpp(results: Dict[str, List[float]], method: str = "minmax"):
    """_normalize_qpp (src/qpp.py:340-374)."""
    import numpy as np
    cols = [[] for _ in range(13)]
    for vals in results.values():
        for i, v in enumerate(vals):
            cols[i].append(v)
    params = []
    for c in cols:
        arr = np.array(c)
        if method == "minmax":
            lo, hi = arr.min(), arr.max()
            params.append((lo, hi - lo if hi > lo else 1.0))
        else:
            params.append((arr.mean(), arr.std() if arr.std() > 0 else 1.0))
    out = {}
    for qid, vals in results.items():
        row = []
        for i, v in enumerate(vals):
            lo, sc = params[i]
            if method == "minmax":
                row.append((v - lo) / sc if sc > 0 else 0.0)
            else:
                row.append((v - lo) / sc)
        out[qid] = row
    return out


def qpp_file_text(results: Dict[str, List[float]]) -> str:
    """The .qpp writer (src/qpp.py:329-335)."""
    lines = []
    for qid in sorted(results.keys(), key=lambda x: int(x) if x.isdigit() else x):
        lines.append(f"{qid}\t" + "\t".join(f"{s:.6f}" for s in results[qid]) + "\n")
    return "".join(lines)


def learned_fusion_from_weights(runs: Dict[str, pd.DataFrame], weights_dict, n_retrievers: int):
    """learned_fusion after the model step, src/fusion.py:436-448, with the same
    pandas calls (row-wise apply, concat, groupby-sum, iterrows)."""
    all_dfs = []
    for ranker, df in runs.items():
        df_copy = df[["qid", "docno", "score"]].copy()
        df_copy["weighted_score"] = df_copy.apply(
            lambda row: row["score"] * weights_dict.get(row["qid"], {}).get(
                ranker, 1.0 / n_retrievers), axis=1)
        all_dfs.append(df_copy[["qid", "docno", "weighted_score"]])
    combined = pd.concat(all_dfs, ignore_index=True)
    aggregated = combined.groupby(["qid", "docno"])["weighted_score"].sum().reset_index()
    fused = defaultdict(list)
    for _, row in aggregated.iterrows():
        fused[row["qid"]].append((row["docno"], row["weighted_score"]))
    return dict(fused)


# ---- research fusion scripts: faithful loops --------------------

def probfuse_pos_to_segment(pos, L, x):
    """ProbFuse.py:30-39."""
    import math
    if pos <= 0:
        pos = 1
    k = math.ceil((pos * x) / float(L))
    if k < 1:
        k = 1
    if k > x:
        k = x
    return int(k)


def train_probfuse(runs_train, qrels_train_dict, x=25, L=100, variant="judged", eps=0.0):
    """ProbFuse.py:92-133, row by row."""
    P_probs = {}
    for ranker, df in runs_train.items():
        rel_counts, nonrel_counts, total_counts = [0] * x, [0] * x, [0] * x
        for qid in sorted(df["qid"].unique()):
            sub = df[df["qid"] == qid]
            for _, row in sub.iterrows():
                k = probfuse_pos_to_segment(int(row["rank"]), L, x) - 1
                doc = str(row["docno"])
                total_counts[k] += 1
                if qid in qrels_train_dict and doc in qrels_train_dict[qid]:
                    if qrels_train_dict[qid][doc] > 0:
                        rel_counts[k] += 1
                    else:
                        nonrel_counts[k] += 1
        probs = [0.0] * x
        for k in range(x):
            if variant.lower() == "all":
                denom, num = total_counts[k], rel_counts[k]
            else:
                denom, num = rel_counts[k] + nonrel_counts[k], rel_counts[k]
            probs[k] = float(num) / float(denom) if denom > 0 else eps
        P_probs[ranker] = probs
    return P_probs


def build_probfuse_run(runs_test, P_probs, x=25, L=100, run_tag="probFuse"):
    """ProbFuse.py:136-187, row by row."""
    from collections import defaultdict
    records = []
    rankers = list(runs_test.keys())
    all_qids = set()
    for r in rankers:
        all_qids.update(runs_test[r]["qid"].unique())
    for qid in sorted(all_qids, key=lambda x: int(x) if x.isdigit() else x):
        doc_scores = defaultdict(float)
        for ranker in rankers:
            df_q = runs_test[ranker][runs_test[ranker]["qid"] == qid]
            for _, row in df_q.iterrows():
                k = probfuse_pos_to_segment(int(row["rank"]), L, x)
                prob = P_probs[ranker][k - 1] if ranker in P_probs else 0.0
                doc_scores[str(row["docno"])] += prob / float(k) if k > 0 else 0.0
        for rank, (docno, score) in enumerate(sorted(doc_scores.items(), key=lambda t: t[1],
                                                     reverse=True), start=1):
            records.append([qid, "Q0", docno, rank, score, run_tag])
    return pd.DataFrame(records, columns=["qid", "iter", "docno", "rank", "score", "runid"])


def build_rrf_run(runs, k=60, qpp_data=None, qpp_method_index=None):
    """QPPrrf_argmax.py:53-76, row by row."""
    from collections import defaultdict
    records = []
    rankers = list(runs.keys())
    for qid in runs[rankers[0]]["qid"].unique():
        doc_scores = defaultdict(float)
        for ranker in rankers:
            df_q = runs[ranker][runs[ranker]["qid"] == int(qid)]
            if df_q.empty:
                continue
            weight = 1.0
            if qpp_data and qpp_method_index is not None:
                try:
                    weight = qpp_data[str(qid)][ranker][qpp_method_index]
                except KeyError:
                    weight = 0.0
            for _, row in df_q.iterrows():
                doc_scores[row["docno"]] += weight * (1.0 / (k + row["rank"]))
        if doc_scores:
            for rank, (docno, score) in enumerate(sorted(doc_scores.items(), key=lambda t: t[1],
                                                         reverse=True), start=1):
                records.append([qid, "Q0", docno, rank, score,
                                "Weighted-RRF" if qpp_data else "RRF"])
    return pd.DataFrame(records, columns=["qid", "iter", "docno", "rank", "score", "runid"])
