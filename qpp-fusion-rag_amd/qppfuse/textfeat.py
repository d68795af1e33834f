"""Text-only QPP inputs: numTerms and the MaxIDF / avgidf proxies.

These are host string operations of QPPBridge.java (numTerms :247-293,
computeMaxIDFProxy :368-380, computeAvgIDFProxy :385-393); the GPU QPP kernel
receives them as per-query arrays (include/qppfuse.h qf_qpp_raw).  Java rules:
toLowerCase(), split("\\s+") with \\s = [ \\t\\n\\x0B\\f\\r] (leading empty token
kept, trailing empty tokens dropped, no match -> [text]), length() in UTF-16
code units, IntStream.average() = (double) sum / count.
"""
from __future__ import annotations

import math
import re
from typing import Iterable, Tuple

import numpy as np

_WS = re.compile(r"[ \t\n\x0b\x0c\r]+")


def split_terms(text: str):
    low = text.lower()
    if not _WS.search(low):
        return [low]
    parts = _WS.split(low)
    while parts and parts[-1] == "":
        parts.pop()
    return parts


def _u16(s: str) -> int:
    return len(s.encode("utf-16-le", "surrogatepass")) // 2


def features(text: str) -> Tuple[int, float, float]:
    terms = split_terms(text)
    uniq = set(terms)
    max_len = max((_u16(t) for t in uniq), default=0)
    max_idf = math.log(1 + len(uniq)) + math.log(1 + max_len) * 0.5
    if terms:
        avg_idf = math.log(1 + sum(_u16(t) for t in terms) / len(terms)) * (len(uniq) / len(terms))
    else:
        avg_idf = math.log(1 + 3.0) * float("nan")
    return len(terms), max_idf, avg_idf


def feature_arrays(texts: Iterable[str]):
    """num_terms int32 [Q], text_feat float64 [Q, 2] for a sequence of query texts."""
    rows = [features(t) for t in texts]
    nt = np.array([r[0] for r in rows], dtype=np.int32)
    tf = np.array([[r[1], r[2]] for r in rows], dtype=np.float64).reshape(-1, 2)
    return nt, tf
