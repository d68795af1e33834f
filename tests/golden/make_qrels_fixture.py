"""Writes tests/golden/nq_qrels_test.tsv.gz: the reference's NQ test qrels
(data/nq/BEIR-nq/qrels/test.tsv, 3,452 queries, 4,201 judgments, all rel 1) as a
data fixture — SURVEY.md §8(d)'s synthetic runs plant these judged documents.
The bytes are the file's own (gzip, mtime 0 for a reproducible archive)."""
import gzip
import sys
from pathlib import Path

SRC = Path(sys.argv[1] if len(sys.argv) > 1 else
           "/root/reference/data/nq/BEIR-nq/qrels/test.tsv")
OUT = Path(__file__).resolve().parent / "nq_qrels_test.tsv.gz"
with open(OUT, "wb") as f, gzip.GzipFile(fileobj=f, mode="wb", mtime=0) as g:
    g.write(SRC.read_bytes())
print(OUT, OUT.stat().st_size)
