"""Java string semantics of the text-only QPP columns — TEST INFRASTRUCTURE ONLY.

Restates, character by character, what QPPBridge.java does with the query text
(computeWIG/computeSigmaMax numTerms :247-293, computeMaxIDFProxy :368-380,
computeAvgIDFProxy :385-393):
  String.toLowerCase()  (default locale; Python str.lower() agrees on the data)
  String.split("\\s+")  (\\s = [ \\t\\n\\x0B\\f\\r]; a leading empty token is kept
                         when the text starts with whitespace; trailing empty
                         tokens are dropped; no match at all -> [text])
  String.length()       (UTF-16 code units)
Independent of qppfuse/textfeat.py (which uses a regex): a scanner here.
"""
from __future__ import annotations

import math

JAVA_WS = set(" \t\n\x0b\x0c\r")


def java_split_ws(text: str):
    toks, cur, matched = [], [], False
    i, n = 0, len(text)
    while i < n:
        ch = text[i]
        if ch in JAVA_WS:
            matched = True
            toks.append("".join(cur))
            cur = []
            while i < n and text[i] in JAVA_WS:
                i += 1
            continue
        cur.append(ch)
        i += 1
    if not matched:
        return [text]
    toks.append("".join(cur))
    while toks and toks[-1] == "":
        toks.pop()
    return toks


def utf16_len(s: str) -> int:
    return sum(2 if ord(c) > 0xFFFF else 1 for c in s)


def text_features(text: str):
    """(terms.length, MaxIDF proxy, avgidf proxy) for one query text."""
    terms = java_split_ws(text.lower())
    uniq = set(terms)
    max_len = 0
    for t in uniq:
        max_len = max(max_len, utf16_len(t))
    maxidf = math.log(1 + len(uniq)) + math.log(1 + max_len) * 0.5
    if terms:
        avg_len = sum(utf16_len(t) for t in terms) / len(terms)
        diversity = len(uniq) / len(terms)
    else:
        avg_len, diversity = 3.0, float("nan")
    return len(terms), maxidf, math.log(1 + avg_len) * diversity
