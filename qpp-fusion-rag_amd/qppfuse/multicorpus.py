"""Several BEIR corpora fused in one batch (BASELINE config C4): namespaced qids.

The reference runs one corpus at a time.  Its two qid sort keys fail on a
mixed batch: write_runfile's `int(x[4:]) if x.startswith("test") else x`
(src/fusion.py:487) and the .qpp writer's `int(x) if x.isdigit() else x`
(src/qpp.py:331) compare int with str as soon as NQ's `test<n>` qids meet
SciFact's numeric or HotpotQA's hex qids (TypeError — kept as is for bare
qids, tests/golden/reference_round2.json "qids.bare_error").

The rule here: a query of corpus C with qid q is `"C:q"` everywhere inside a
multi-corpus batch — packing, fusion, .qpp data and run files.  No namespaced
qid is all digits or starts with "test" (corpus names are lower-case
identifiers other than "test..."), so both reference keys reduce to plain
string order, the reference's own behaviour on these strings (pinned:
"qids.namespaced_order"), and corpora form contiguous blocks in name order.
Splitting a batch back (split_fused / write_runfiles_per_corpus) restores the
bare qids, and each corpus's run file is byte-identical to the file the
reference writes for that corpus alone (its per-corpus order: pinned by
"qids.per_corpus_order").

Packing is per corpus with the native loader; the run sets are then
concatenated (corpus blocks in namespace order are already in sorted-qid
order, so no query moves) with docnos offset per corpus — a query only holds
documents of its own corpus, so the within-query docno order the evaluation
and learned fusion rely on is kept.
"""
from __future__ import annotations

import re
from typing import Dict, List, Mapping, Optional, Sequence, Tuple

import numpy as np
import pandas as pd

from .runset import RunSet

SEP = ":"
_NAME = re.compile(r"^[a-z][a-z0-9_\-]*$")


def check_corpus_name(name: str) -> str:
    if not _NAME.match(name) or name.startswith("test") or SEP in name:
        raise ValueError(f"corpus name {name!r}: use a lower-case identifier not starting "
                         f"with 'test' (it prefixes qids as '<corpus>{SEP}<qid>')")
    return name


def namespace_qid(corpus: str, qid: str) -> str:
    return f"{corpus}{SEP}{qid}"


def split_qid(nsqid: str) -> Tuple[str, str]:
    corpus, sep, qid = nsqid.partition(SEP)
    if not sep:
        raise ValueError(f"qid {nsqid!r} is not namespaced ('<corpus>{SEP}<qid>')")
    return corpus, qid


def _concat_runsets(parts: Sequence[Tuple[str, RunSet]]) -> RunSet:
    rankers = parts[0][1].rankers
    for c, rs in parts[1:]:
        if rs.rankers != rankers:
            raise ValueError(f"corpus {c!r} has rankers {rs.rankers}, expected {rankers} "
                             "(the same run files, in the same order, for every corpus)")
    qids, docnos, offs, docid, score, rank, micro = [], [], [], [], [], [], []
    e0 = d0 = 0
    use_micro = all(rs.micro is not None for _, rs in parts)
    for c, rs in parts:
        qids += [namespace_qid(c, q) for q in rs.qids]
        docnos.append(np.asarray(rs.docnos, dtype=object))
        offs.append(rs.list_off[:-1] + e0)
        docid.append(rs.docid.astype(np.uint64) + d0)
        score.append(rs.score)
        rank.append(rs.rank)
        if use_micro:
            micro.append(rs.micro)
        e0 += rs.n_entries
        d0 += len(rs.docnos)
    if d0 >= 0xFFFFFFFF:
        raise ValueError("too many distinct docnos for uint32 ids")
    out = RunSet(qids=qids, rankers=list(rankers), docnos=np.concatenate(docnos),
                 list_off=np.concatenate(offs + [np.array([e0], np.int64)]),
                 docid=np.concatenate(docid).astype(np.uint32), score=np.concatenate(score),
                 rank=np.concatenate(rank), micro=np.concatenate(micro) if use_micro else None)
    out.rank_is_position = all(rs.rank_is_position for _, rs in parts)
    out.canonical = all(rs.canonical for _, rs in parts)
    out.has_dups = any(rs.has_dups for _, rs in parts)
    return out


def load_runs(runs_dirs: Mapping[str, str], use_normalized: bool = True
              ) -> Dict[str, pd.DataFrame]:
    """{corpus: runs_dir} -> {ranker: DataFrame} with namespaced qids (the fusion
    module's load_runs per corpus, src/fusion.py:46-76).  The packed run set is
    cached for the returned frames, like fusion.load_runs."""
    from . import fastio, fusion
    import os
    # namespace order: "<corpus>:" prefixes sort as the corpora's blocks
    corpora = sorted((check_corpus_name(c) for c in runs_dirs), key=lambda c: c + SEP)
    suffix = ".norm.res" if use_normalized else ".res"
    parts, frames_by = [], {}
    names0 = None
    for c in corpora:
        d = runs_dirs[c]
        files = [f for f in os.listdir(d) if f.endswith(suffix)]
        if not files:
            raise FileNotFoundError(f"No {suffix} files found in {d}")
        names = [f.replace(suffix, "") for f in files]
        if names0 is None:
            names0 = names
        elif sorted(names) != sorted(names0):
            raise ValueError(f"corpus {c!r} has rankers {names}, expected {names0}")
        files = [files[names.index(n)] for n in names0]  # the first corpus's run order
        rs, frames = fastio.parse_runs([os.path.join(d, f) for f in files], names0)
        parts.append((c, rs))
        frames_by[c] = frames
    rs = _concat_runsets(parts)
    out = {}
    for r in names0:
        pieces = []
        for c in corpora:
            df = frames_by[c][r].copy(deep=False)
            df["qid"] = namespace_qid(c, "") + df["qid"].astype(object)
            pieces.append(df)
        out[r] = pd.concat(pieces, ignore_index=True)
    fusion._remember(out, rs)
    return out


def load_qpp_scores(qpp_dirs: Mapping[str, str]) -> Dict[str, Dict[str, List[float]]]:
    """{corpus: qpp_dir} -> {"<corpus>:<qid>": {retriever: [13 floats]}}."""
    from .data_utils import load_qpp_scores as load_one
    out = {}
    for c in sorted(qpp_dirs, key=lambda c: c + SEP):
        check_corpus_name(c)
        for q, v in load_one(qpp_dirs[c]).items():
            out[namespace_qid(c, q)] = v
    return out


def split_fused(fused: Mapping[str, list]) -> Dict[str, Dict[str, list]]:
    """{"<corpus>:<qid>": list} -> {corpus: {qid: list}} (corpus order, then batch order)."""
    out: Dict[str, Dict[str, list]] = {}
    for nq in fused.keys():
        c, q = split_qid(nq)
        out.setdefault(c, {})[q] = fused[nq]
    return out


def write_runfiles_per_corpus(fused, paths: Mapping[str, str], tag: str = "fusion") -> None:
    """One run file per corpus with the bare qids — the bytes the reference's
    write_runfile (src/fusion.py:480-492) writes for that corpus alone."""
    from . import fusion
    if isinstance(fused, fusion.FusedRun) and fused._rs is not None:
        for c, path in paths.items():
            pre = c + SEP
            fusion.write_fused_native(fused, path, tag, select=lambda q: q.startswith(pre),
                                      rename=lambda q: q[len(pre):] if q.startswith(pre) else q)
            print(f"Wrote fused run to {path}")
        return
    per = split_fused(fused)
    for c, path in paths.items():
        fusion.write_runfile(per.get(c, {}), path, tag)


def batch_qids(qids_by_corpus: Mapping[str, Sequence[str]]) -> List[str]:
    """The namespaced qids of a batch in its packed (= sorted string) order."""
    return sorted(namespace_qid(check_corpus_name(c), q)
                  for c, qs in qids_by_corpus.items() for q in qs)
