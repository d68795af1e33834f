#!/usr/bin/env python3
"""Benchmark: fused queries/sec of the fusion + QPP hot path on MI355X.

Workload (BASELINE.json configs[1], "C2"): BEIR-NQ-shaped batches of 3,452
queries per GPU x 5 retrievers x top-1000, synthetic lists generated on device
(DESIGN.md "Synthetic runs"); one step = the whole path for the batch, with the
inputs already resident in HBM:
  1. per-query min-max of every list -> the .norm.res values (micro-units)
  2. 13 QPP predictors per (query, retriever) list (top_k = 100, k = 50)
  3. per-column min/max of the predictors (+ RCCL MIN all-reduce when N > 1)
  4. normalise all 13 columns + "%.6f" (the .qpp table, src/qpp.py:324-372) and the
     RSD weight per (query, retriever) — inside the fusion launch (qf_fuse_qpp_micro)
  5. all six fusions (CombSUM, CombMNZ, RRF, W-CombSUM, W-CombMNZ, W-RRF) of
     every query, full fused lists sorted (what write_runfile needs).
Queries shard across ranks (weak scaling); the only collective is the 1 KB
all-reduce of step 3.  Rank 0 prints ONE JSON line.

python bench.py [--gpus N] [--steps K] [--warmup W]
For N > 1 one process per GPU: either the driver launches this script under
torch.distributed.run (WORLD_SIZE set), or — run plainly as
`python bench.py --gpus N` — this process, before it makes any GPU call,
starts `torch.distributed.run --nproc-per-node N` on itself as a child and exits
with its code.  For N > 1 the timed step includes the north star's collective:
every rank's fused top-k (default 100) gathered to rank 0 over RCCL, pipelined:
step i's gather runs on the communicator's stream beside step i+1's kernels (the
last one is waited for inside the timed region).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
for _p in (ROOT, ROOT / "qpp-fusion-rag_amd"):
    if str(_p) not in sys.path:
        sys.path.insert(0, str(_p))

import numpy as np  # noqa: E402
import torch  # noqa: E402

METHODS = ["combsum", "combmnz", "rrf", "wcombsum", "wcombmnz", "wrrf"]
NAMES = ["BGE", "BM25", "BM25_MonoT5", "BM25_TCT", "Splade", "R5", "R6", "R7"]
# BASELINE.json configs (SURVEY.md §8 shorthand).  The default run — and the
# driver's — is C2; the others measure the remaining configs' hot paths.
WORKLOADS = {
    "c1": dict(queries=3452, total=False, methods=["combsum", "rrf"], qpp=False, qpp_index=5,
               retrievers=3, k=100,
               desc="C1: BEIR-NQ-shaped, 3452 queries/GPU x 3 retrievers (BM25/BGE/SPLADE) x "
                    "top-100; min-max + CombSUM + RRF, full sorted lists"),
    "c2": dict(queries=3452, total=False, methods=METHODS, qpp=True, qpp_index=5,
               desc="C2: BEIR-NQ-shaped, 3452 queries/GPU x 5 retrievers x top-1000; "
                    "min-max + QPP(13) + 6 fusions, full sorted lists"),
    "c3": dict(queries=1_000_000, total=True, methods=["combsum", "rrf"], qpp=False,
               qpp_index=5,
               desc="C3: synthetic 1M queries in all x 5 retrievers x top-1000, query-sharded; "
                    "min-max + CombSUM + RRF, full sorted lists"),
    "c4": dict(queries=11157, total=True, methods=["wcombsum"], qpp=True, qpp_index=-1,
               desc="C4: HotpotQA+SciFact+NQ-shaped, 11157 queries in all x 5 x top-1000; "
                    "min-max + QPP(13) + W-CombSUM with the mean of the 13 columns"),
    "c5": dict(queries=3452, total=False, methods=["learned"], qpp=True, qpp_index=5,
               desc="C5: C2 + learned fusion with the reference's NQ MultiOutput-LightGBM "
                    "(tests/golden/lgbm fixture): min-max + QPP(13) + GBDT weights + fusion"),
}
HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md), 6.3 TB/s measured copy
SEED = 20251212


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--gather-topk", type=int, default=None,
                    help="per step, gather every rank's fused top-k to rank 0 over RCCL "
                         "(default: 100 when N > 1, else 0; 0 = fused lists stay on their "
                         "rank, as each rank writes its own qid range).  Bytes into rank 0 "
                         "per step: N x queries x methods x k x 12 (C2 weak-scaled, k 100: "
                         "24.9 MB per rank, 174 MB from 7 peers at N = 8 — ~290 GB/s at a "
                         "0.6 ms step, against rank 0's 7 x ~50 GB/s practical xGMI ingress: "
                         "DESIGN.md §7); the N > 1 line reports the bytes, the host time in "
                         "the gather's wait and the step without the gather")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="put every rank on GPU 0 (use with --dist-backend gloo)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--queries", type=int, default=None,
                    help="queries per GPU (default: the workload's; C3/C4 split their total)")
    ap.add_argument("--retrievers", type=int, default=None)
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--qpp-top-k", type=int, default=100)
    ap.add_argument("--qpp-index", type=int, default=None)
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="queries per CPU-baseline process timed through the Python port of "
                         "the reference (0 = skip; default: the workload's — C2's 125 x 16 "
                         "processes are SURVEY §8(d)'s 2,000-query sample, ~50 s)")
    ap.add_argument("--cpu-workers", type=int, default=None,
                    help="processes the CPU baseline runs on (default min(16, cpu_count))")
    ap.add_argument("--native-sample", type=int, default=400,
                    help="queries timed through the C oracle (0 = skip)")
    ap.add_argument("--check", type=int, default=8, help="queries checked bit-exact vs oracle")
    ap.add_argument("--ndcg-sample", type=int, default=1000,
                    help="queries whose NDCG@10 is recomputed on the CPU reference path")
    ap.add_argument("--generator", choices=["nq", "legacy"], default="nq",
                    help="synthetic runs: nq = SURVEY.md §8(d) (qf_synth_runs_nq: 2K shared pool "
                         "at p 0.5 + the 2,681,468-id NQ pool, Gamma / Beta / ln-Beta scores, the "
                         "real NQ test qrels planted at Geometric(0.15) ranks); legacy = rounds "
                         "1-4's exp-decay generator (qf_synth_runs)")
    a = ap.parse_args()
    a.wl = WORKLOADS[a.workload]
    if a.qpp_index is None:
        a.qpp_index = a.wl["qpp_index"]
    a.methods = list(a.wl["methods"])
    if a.retrievers is None:
        a.retrievers = a.wl.get("retrievers", 5)
    if a.k is None:
        a.k = a.wl.get("k", 1000)
    return a


_NQ_QRELS = None


def nq_qrels():
    """The reference's NQ test qrels (tests/golden/nq_qrels_test.tsv.gz, a data fixture of
    data/nq/BEIR-nq/qrels/test.tsv): CSR over test0 .. test3451 of corpus ids (doc{n} ->
    n); every judgment is rel 1."""
    global _NQ_QRELS
    if _NQ_QRELS is None:
        import gzip
        rows = gzip.decompress((ROOT / "tests" / "golden" / "nq_qrels_test.tsv.gz")
                               .read_bytes()).decode().splitlines()[1:]
        per = {}
        for line in rows:
            q, d, _ = line.split("\t")
            per.setdefault(int(q[4:]), []).append(int(d[3:]))
        n = max(per) + 1
        off = np.zeros(n + 1, np.int64)
        off[1:] = np.cumsum([len(per.get(q, ())) for q in range(n)])
        doc = np.array([d for q in range(n) for d in per.get(q, ())], np.uint32)
        _NQ_QRELS = (off, doc)
    return _NQ_QRELS


def gen_runs(args, q_begin: int, Q: int, R: int, K: int):
    """The bench's synthetic runs on device: (list_off, docid, raw score)."""
    from qppfuse import engine
    if args.generator == "nq":
        qo, qd = nq_qrels()
        return engine.synth_runs_nq(q_begin, Q, R, K, qo, qd, seed=SEED)
    return engine.synth_runs(q_begin, Q, R, K, seed=SEED)


def launch_ranks(args, script=None, argv=None) -> int:
    """`--gpus N` without a launcher: run torch.distributed.run on this script as a
    child process (this process has made no GPU call) and return its exit code."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={port}", str(script or Path(__file__).resolve())] + \
        list(sys.argv[1:] if argv is None else argv)
    env = dict(os.environ, QPPFUSE_BENCH_LAUNCHED="1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    progress(f"launching {args.gpus} ranks: {' '.join(cmd[1:6])} ...")
    return subprocess.run(cmd, env=env).returncode


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch with "
                         f"torch.distributed.run --nproc-per-node {args.gpus} (or without a "
                         f"launcher: python bench.py --gpus {args.gpus})")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.rehearse_one_gpu:  # N-rank rehearsal on a 1-GPU box (gloo): all ranks on GPU 0
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":  # RCCL over xGMI
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
    return world, rank, torch.device("cuda", local)


def c4_queries():
    """C4's 11,157 namespaced qids in batch order and their query texts."""
    import gzip
    from qppfuse import multicorpus
    g = ROOT / "tests" / "golden"
    bq = json.loads(gzip.decompress((g / "beir_qids.json.gz").read_bytes()))
    text = {}
    for ds in ("nq", "scifact"):
        fx = json.loads((g / f"qpp_textcols_{ds}.json").read_text())
        text.update({multicorpus.namespace_qid(ds, q): t for q, t in zip(fx["qids"], fx["text"])})
    qids = multicorpus.batch_qids(bq)
    return qids, [text.get(q, multicorpus.split_qid(q)[1]) for q in qids]


def text_inputs(q_begin, Q):
    """Deterministic per-query numTerms and text-feature columns (host, tiny)."""
    rng = np.random.default_rng([SEED, 99, q_begin])
    nt = rng.integers(2, 15, Q).astype(np.int32)
    tf = np.stack([np.log1p(nt) + 0.5 * np.log1p(rng.integers(3, 14, Q)),
                   np.log1p(rng.uniform(3, 9, Q)) * rng.uniform(0.6, 1.0, Q)], 1)
    return nt, tf


class Pipeline:
    def __init__(self, args, world, rank, dev):
        from qppfuse import engine
        self.engine = engine
        self.args, self.world, self.rank, self.dev = args, world, rank, dev
        R, K = args.retrievers, args.k
        wl = args.wl
        self.plan = None
        if args.queries is not None:
            Q, self.q_begin = args.queries, rank * args.queries
        elif wl["total"]:  # strong scaling: the workload's total split across ranks,
            # balanced by Σ entries; every rank derives the same plan from
            # the run set's list offsets (the synthetic lists are K long each)
            from qppfuse.dist import shard_by_entries
            n = wl["queries"] * R
            self.plan = shard_by_entries(np.arange(n + 1, dtype=np.int64) * K, R, world)
            Q, self.q_begin = int(self.plan[rank + 1] - self.plan[rank]), int(self.plan[rank])
        else:
            Q, self.q_begin = wl["queries"], rank * wl["queries"]
        self.Q, self.R, self.K = Q, R, K
        if self.plan is None:
            self.shard_sizes = [Q] * world
        else:
            self.shard_sizes = [int(x) for x in np.diff(self.plan)]
        self.methods = args.methods
        self.off, self.docid, self.raw = gen_runs(args, self.q_begin, Q, R, K)
        self.qids = None
        if args.workload == "c4" and args.queries is None:
            self.qids = c4_queries()[0][self.q_begin:self.q_begin + Q]
        nt, tf = self.text_arrays(self.q_begin, Q)
        self.nt = torch.from_numpy(nt).to(dev)
        self.tf = torch.from_numpy(tf).to(dev)
        E = Q * R * K
        self.micro = torch.empty(E, dtype=torch.int32, device=dev)
        self.qraw = torch.empty((Q * R, 13), dtype=torch.float64, device=dev)
        self.mm = torch.empty(2 * R * 13, dtype=torch.float64, device=dev)
        # the .qpp table of the batch (every list's 13 "%.6f" values, src/qpp.py:324-334):
        # written by the join (qf_fuse_qpp_micro) or the normalisation launch
        self.qmicro = torch.empty(Q * R * 13, dtype=torch.int64, device=dev)
        self.out = engine.alloc_fuse_out(Q, E, engine.methods_mask(self.methods), dev)
        self.w = None
        if "learned" in self.methods:
            from qppfuse import lgbm
            model = lgbm.load_fusion_model(ROOT / "tests" / "golden" / "lgbm" /
                                           "nq_fusion_multioutput.json.gz")
            self.packed = lgbm.pack_model(model)
            names = NAMES[:R]
            # X columns: model.retrievers order, 13 QPP values each (src/fusion.py:421-427)
            self.block_runs = [names.index(r) if r in names else -1 for r in model.retrievers]
            self.X = torch.empty((Q, 13 * len(model.retrievers)), dtype=torch.float64, device=dev)
            self.run_to_booster = [model.retrievers.index(n) if n in model.retrievers else -1
                                   for n in names]
        self.ev = []
        self.pending = None  # the previous step's top-k gather (dist.TopkGather handle)
        self.wait_s = 0.0    # host seconds rank 0 spends in the gathers' wait() (timed steps)
        self.timed_steps = 0
        self.gather, self.n_step, self.gathered = None, 0, None
        if world > 1 and args.gather_topk > 0:  # every buffer of the gather, made once
            from qppfuse.dist import TopkGather
            self.gather = TopkGather(self.shard_sizes, len(self.methods), args.gather_topk, dev,
                                     dst=0)
        torch.cuda.synchronize()

    def shard_begin(self, r: int) -> int:
        """First global query of rank r's shard (as __init__ computes its own)."""
        if self.plan is None:
            return r * self.shard_sizes[r]
        return int(self.plan[r])

    def text_arrays(self, q_begin: int, Q: int):
        """numTerms / text-feature columns of the shard [q_begin, q_begin + Q)."""
        if self.args.workload == "c4" and self.args.queries is None:
            # the real test qids of HotpotQA + SciFact + NQ, namespaced (qppfuse.multicorpus),
            # in batch order; query texts as compute_qpp_for_res_file gets them
            # (queries.jsonl; HotpotQA's is an LFS pointer, so its qid, src/qpp.py:312)
            from qppfuse import textfeat
            return textfeat.feature_arrays(c4_queries()[1][q_begin:q_begin + Q])
        return text_inputs(q_begin, Q)

    def fuse_block(self, q_begin: int, Q_shard: int, start: int, n: int):
        """Queries [start, start + n) of the shard beginning at global query q_begin
        (of Q_shard queries), regenerated from the counter-based generator and run
        through this step's kernels with the step's QPP min / max (after the
        all-reduce: every rank normalises with the same global values)."""
        e, a, R, K = self.engine, self.args, self.R, self.K
        off, docid, raw = gen_runs(a, q_begin + start, n, R, K)
        _, micro = e.minmax_per_query(raw, off, want_norm=False)
        w, qppw = None, None
        if a.wl["qpp"]:
            nt, tf = self.text_arrays(q_begin, Q_shard)
            nt = torch.from_numpy(np.ascontiguousarray(nt[start:start + n])).to(self.dev)
            tf = torch.from_numpy(np.ascontiguousarray(tf[start:start + n])).to(self.dev)
            qraw = e.qpp_raw(raw, off, R, a.qpp_top_k, nt, tf)
            if "learned" in self.methods:
                w = e.learned_gbdt_weights(None, n, R, self.block_runs, self.packed,
                                           self.run_to_booster, raw_qpp=qraw, mm=self.mm,
                                           list_off=off)
            elif a.qpp_index >= 0:
                qppw = (qraw, self.mm, "minmax", a.qpp_index)
            else:
                w = e.qpp_normalize(qraw, self.mm, off, R, "minmax", a.qpp_index,
                                    want_micro=False)["weights"]
        out = e.fuse(off, docid, micro, R, self.methods, 60, weights=w, max_entries=R * K,
                     qpp=qppw)
        return e.fused_topk(out, off, R, a.gather_topk)

    def gather_parity(self, per_block: int = 4):
        """Rank 0: the gathered top-k rows of EVERY rank checked byte for byte against
        rows rank 0 recomputes itself — each shard's first and last `per_block`
        queries regenerated (qf_synth_runs is counter-based in the global query id)
        and fused here.  None off rank 0 or without a gather."""
        if self.gather is None or self.rank != 0 or self.gathered is None:
            return None
        ok, checked = True, 0
        for r, (gd, gs) in enumerate(self.gathered):
            n_r = self.shard_sizes[r]
            q0 = self.shard_begin(r)
            for start in sorted({0, max(0, n_r - per_block)}):
                n = min(per_block, n_r - start)
                if n <= 0:
                    continue
                d, sc = self.fuse_block(q0, n_r, start, n)
                ok &= bool(torch.equal(gd[start:start + n].to(self.dev), d))
                ok &= bool(torch.equal(gs[start:start + n].to(self.dev).view(torch.int64),
                                       sc.view(torch.int64)))
                checked += n
        return {"ranks": len(self.gathered), "queries_checked": checked, "bit_exact": ok,
                "how": "rank 0 regenerates the first and last queries of every rank's shard "
                       "(counter-based generator), fuses them with the step's kernels and "
                       "compares the gathered top-k rows byte for byte"}

    def step(self, timed=False):
        from qppfuse import _lib
        e, a = self.engine, self.args
        s = torch.cuda.current_stream().cuda_stream
        minmax = lambda: _lib.call("qf_minmax_per_query", self.raw.data_ptr(),
                                   self.off.data_ptr(), self.Q * self.R, None,
                                   self.micro.data_ptr(), s)
        w, qppw = None, None
        if not a.wl["qpp"]:
            minmax()
        else:
            e.qpp_raw(self.raw, self.off, self.R, a.qpp_top_k, self.nt, self.tf, out=self.qraw)
            if self.world > 1:
                e.qpp_colminmax(self.qraw, self.off, self.R, out=self.mm)
                # the path's only exchange: ~1 KB over RCCL/xGMI, hidden behind the
                # min-max kernel
                from qppfuse.dist import allreduce_minmax
                work = allreduce_minmax(self.mm, async_op=True)
                minmax()
                work.wait()
            else:  # every query here: the column extremes and the min-max in one launch
                e.minmax_colminmax(self.raw, self.off, self.R, self.qraw, micro_out=self.micro,
                                   mm_out=self.mm)
            if "learned" in self.methods:
                # the .qpp values as features (normalised on the fly from the raw
                # predictors and the column statistics), GBDT, weights: one launch
                w = e.learned_gbdt_weights(None, self.Q, self.R, self.block_runs, self.packed,
                                           self.run_to_booster, raw_qpp=self.qraw, mm=self.mm,
                                           list_off=self.off)
            elif a.qpp_index >= 0:  # one column: the W-* weights inside the fusion (qf_fuse_qpp)
                qppw = (self.qraw, self.mm, "minmax", a.qpp_index)
            else:  # the mean of 13 columns per list: the normalisation launch (qf_fuse_qpp
                # would put 13 normalisations per list on the join's start; C4: 0.665 ->
                # 0.73 ms per step)
                nz = e.qpp_normalize(self.qraw, self.mm, self.off, self.R, "minmax",
                                     a.qpp_index, want_micro=True)
                w, self.qmicro = nz["weights"], nz["micro"]
        if timed:
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
        e.fuse(self.off, self.docid, self.micro, self.R, self.methods, 60, weights=w,
               max_entries=self.R * self.K, out=self.out, qpp=qppw,
               qpp_micro_out=self.qmicro if qppw is not None else None)
        if timed:
            t1.record()
            self.ev.append((t0, t1))
        if self.gather is not None and a.gather_topk > 0:  # the fused top-k onto rank 0 (RCCL)
            # pipelined: this step's gather runs on the communicator's stream beside
            # the next step's kernels; the previous step's is waited for here, after
            # this step's kernels are queued.  Two buffer sets alternate: the top-k
            # kernel writes this step's rows straight into set n % 2 (no pad, no cat)
            if self.pending is not None:
                tw = time.perf_counter()
                self.gathered = self.pending.wait()
                if timed:
                    self.wait_s += time.perf_counter() - tw
            if timed:
                self.timed_steps += 1
            e.fused_topk(self.out, self.off, self.R, a.gather_topk,
                         dest=self.gather.buffers(self.n_step))
            self.pending = self.gather.start(self.n_step)
            self.n_step += 1
        self.w = w

    def drain(self):
        """The last step's gather, before the timed region's final synchronize."""
        if self.pending is not None:
            tw = time.perf_counter()
            self.gathered = self.pending.wait()
            self.wait_s += time.perf_counter() - tw
            self.pending = None

    def fuse_kernel_ms(self):
        return float(np.mean([a.elapsed_time(b) for a, b in self.ev]))

    def fuse_bytes(self):
        """Algorithmic HBM bytes of one qf_fuse launch."""
        uc = self.out.union_count.cpu().numpy()[:self.Q].astype(np.int64)
        N = self.Q * self.R * self.K
        M = len(self.methods)
        weighted = any(m.startswith("w") or m == "learned" for m in self.methods)
        reads = N * (4 + 4) + (self.Q * self.R * 8 if weighted else 0) + (self.Q * self.R + 1) * 8
        writes = int(uc.sum()) * (4 + M * (2 + 8)) + self.Q * 4
        if self.args.wl["qpp"] and self.args.qpp_index >= 0 and "learned" not in self.methods:
            # qf_fuse_qpp_micro: the raw predictors in, the .qpp micro-units out
            reads += self.Q * self.R * 13 * 8
            writes += self.Q * self.R * 13 * 8
        return reads + writes, float(uc.mean())


def synth_qrels(q_begin: int, Q: int, K: int, generator: str = "nq"):
    """Judged documents of the synthetic queries (qrel_off, docid, rel).  nq: query q's
    are the NQ test judgments of test{q mod 3452} (the documents qf_synth_runs_nq
    planted), rel 1.  legacy: 1-3 pool documents each (the first rel 2, the others rel
    1) — ids as qf_synth_runs draws pool documents."""
    if generator == "nq":
        off, doc = nq_qrels()
        qq = np.arange(q_begin, q_begin + Q, dtype=np.int64) % (len(off) - 1)
        n = off[qq + 1] - off[qq]
        qo = np.zeros(Q + 1, np.int64)
        qo[1:] = np.cumsum(n)
        idx = np.repeat(off[qq], n) + (np.arange(qo[-1]) - np.repeat(qo[:-1], n))
        return qo, doc[idx].astype(np.uint32), np.ones(int(qo[-1]), np.int32)
    qg = np.arange(q_begin, q_begin + Q, dtype=np.int64)
    nrel = 1 + qg % 3
    qo = np.zeros(Q + 1, np.int64)
    qo[1:] = np.cumsum(nrel)
    rep = np.repeat(qg, nrel)
    pidx = np.arange(qo[-1]) - np.repeat(qo[:-1], nrel)
    qd = ((rep * K + pidx) & 0x7FFFFFFF).astype(np.uint32)
    qr = np.where(pidx == 0, 2, 1).astype(np.int32)
    return qo, qd, qr


def ndcg_device(p: Pipeline):
    """NDCG@10 of every fused run on device (qf_eval, scores as the .res text)."""
    from qppfuse.evaluation import evaluate_device
    qo, qd, qr = synth_qrels(p.q_begin, p.Q, p.K, p.args.generator)
    t = lambda a: torch.from_numpy(a).to(p.dev)
    qdev = (t(qo), t(qd.view(np.int32)), t(qr))
    o = p.out
    run = lambda: evaluate_device(p.off, p.R, o.union_count, o.union_docid, o.perm, o.fused,
                                  o.fused.shape[1], len(p.methods), p.Q, qdev,
                                  int(np.diff(qo).max()), ["nDCG@10"], text_scores=True)
    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    vals = run()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    return vals[:, :, 0].cpu().numpy(), ms


def ndcg_delta(p: Pipeline, dev_vals, nq: int):
    """NDCG@10 of the CPU reference path (C oracle fusion + trec_eval restatement)
    on the first nq queries vs the device values: largest |delta|."""
    from oracle import _loader as coracle
    h = host_sample(p, nq)
    sc = h["micro"].astype(np.float64) / 1e6
    qo, qd, qr = synth_qrels(p.q_begin, nq, p.K, p.args.generator)
    worst_q, worst_mean = 0.0, 0.0
    for m, name in enumerate(p.methods):
        if name not in METHODS:
            continue
        ud_all, uc, perm, fused = coracle.fuse(h["off"], h["docid"], sc, p.R, name, 60,
                                               weights=h["w"])
        roff = np.zeros(nq + 1, np.int64)
        roff[1:] = np.cumsum(uc)
        b = h["off"][:-1:p.R][:nq]
        rdoc = np.concatenate([ud_all[b[q] + perm[b[q]:b[q] + uc[q]].astype(np.int64)]
                               for q in range(nq)])
        rsc = np.concatenate([fused[b[q]:b[q] + uc[q]] for q in range(nq)])
        ref = coracle.evaluate(roff, rdoc, rsc, qo, qd, qr, ["nDCG@10"], text=True)[:, 0]
        d = dev_vals[m, :nq]
        worst_q = max(worst_q, float(np.nanmax(np.abs(d - ref))))
        worst_mean = max(worst_mean, abs(float(np.nanmean(d)) - float(np.nanmean(ref))))
    return worst_q, worst_mean


def ndcg_delta_learned(p: Pipeline, dev_vals, nq: int):
    """C5: NDCG@10 of learned fusion on the CPU reference path vs the device values —
    the 13 predictors of every list of the batch by the Java restatement
    (oracle/qpp_oracle.c), min-max per retriever column over the batch and "%.6f"
    (src/qpp.py:340-374, 329-335), the features in the model's retriever order, the
    LightGBM walk restated (oracle/lgbm_oracle.py), the weighted groupby-sum as pandas'
    Kahan sum in run order (src/fusion.py:436-446), the trec_eval restatement."""
    from oracle import _loader as coracle
    from oracle import lgbm_oracle
    from qppfuse import lgbm
    R, K, Q = p.R, p.K, p.Q
    off_all = p.off.cpu().numpy()
    raw_all = p.raw[: off_all[-1]].cpu().numpy()
    cut = [raw_all[off_all[l]:off_all[l + 1]][: p.args.qpp_top_k or None] for l in range(Q * R)]
    coff = np.zeros(Q * R + 1, np.int64)
    coff[1:] = np.cumsum([len(c) for c in cut])
    nt, tf = p.nt.cpu().numpy(), p.tf.cpu().numpy()
    qraw = coracle.qpp_raw(np.concatenate(cut), coff, np.repeat(nt, R), np.repeat(tf[:, 0], R),
                           np.repeat(tf[:, 1], R))
    feats = np.zeros((Q * R, 13))
    for r in range(R):  # one .qpp file per retriever: min-max over its queries, "%.6f"
        col = qraw[r::R]
        lo, hi = col.min(axis=0), col.max(axis=0)
        sc = np.where(hi > lo, hi - lo, 1.0)
        feats[r::R] = np.array([[float(f"{v:.6f}") for v in row] for row in (col - lo) / sc])
    model = lgbm.load_fusion_model(ROOT / "tests" / "golden" / "lgbm" /
                                   "nq_fusion_multioutput.json.gz")
    names = NAMES[:R]
    X = np.zeros((nq, 13 * len(model.retrievers)))
    for j, rn in enumerate(model.retrievers):
        if rn in names:
            X[:, 13 * j:13 * j + 13] = feats[names.index(rn)::R][:nq]
    pred = lgbm_oracle.model_predict(model, X)
    w = np.array([[pred[q, model.retrievers.index(n)] if n in model.retrievers else 1.0 / len(model.retrievers)
                   for n in names] for q in range(nq)])
    h = host_sample(p, nq)
    sc = h["micro"].astype(np.float64) / 1e6
    qo, qd, qr = synth_qrels(p.q_begin, nq, p.K, p.args.generator)
    roff, rdoc, rsc = [0], [], []
    for q in range(nq):
        ent_d, ent_v = [], []
        for r in range(R):  # pandas concat order: run by run, row by row
            a, b = h["off"][q * R + r], h["off"][q * R + r + 1]
            ent_d.append(h["docid"][a:b])
            ent_v.append(sc[a:b] * w[q, r])
        d = np.concatenate(ent_d)
        v = np.concatenate(ent_v)
        order = np.argsort(d, kind="stable")  # each document's terms in run order
        d, v = d[order], v[order]
        first = np.r_[True, d[1:] != d[:-1]]
        g = np.cumsum(first) - 1
        pos = np.arange(len(d)) - np.flatnonzero(first)[g]
        acc = np.zeros(g[-1] + 1)
        comp = np.zeros(g[-1] + 1)
        for t in range(int(pos.max()) + 1):  # Kahan, one term of every document at a time
            m = pos == t
            y = v[m] - comp[g[m]]
            tt = acc[g[m]] + y
            c = (tt - acc[g[m]]) - y
            comp[g[m]] = np.where(np.isnan(c), 0.0, c)
            acc[g[m]] = tt
        rdoc.append(d[first])
        rsc.append(acc)
        roff.append(roff[-1] + len(acc))
    ref = coracle.evaluate(np.array(roff, np.int64), np.concatenate(rdoc),
                           np.concatenate(rsc), qo, qd, qr, ["nDCG@10"], text=True)[:, 0]
    dv = dev_vals[p.methods.index("learned"), :nq]
    return (float(np.nanmax(np.abs(dv - ref))),
            abs(float(np.nanmean(dv)) - float(np.nanmean(ref))))


def host_sample(p: Pipeline, nq: int):
    """Copy the first nq queries' inputs + device outputs to host numpy.  When the
    step's fusion took its W-* weights from the QPP predictors (qf_fuse_qpp), `w` is
    what qf_qpp_normalize gives for the same predictors and column statistics — the
    oracle then fuses with those, so the check covers the in-kernel weights too."""
    R, K = p.R, p.K
    n = nq * R * K
    off = p.off[: nq * R + 1].cpu().numpy()
    w = p.w
    if w is None and p.args.wl["qpp"] and "learned" not in p.methods:
        w = p.engine.qpp_normalize(p.qraw, p.mm, p.off, R, "minmax", p.args.qpp_index,
                                   want_micro=False)["weights"]
    return dict(off=off, docid=p.docid[:n].cpu().numpy().view(np.uint32),
                raw=p.raw[:n].cpu().numpy(), micro=p.micro[:n].cpu().numpy(),
                w=None if w is None else w[: nq * R].cpu().numpy(),
                nt=p.nt[:nq].cpu().numpy(),
                tf=p.tf[:nq].cpu().numpy(), qraw=p.qraw[: nq * R].cpu().numpy())


def check_parity(p: Pipeline, nq: int):
    from oracle import _loader as coracle
    h = host_sample(p, nq)
    sc = h["micro"].astype(np.float64) / 1e6
    uc = p.out.union_count[:nq].cpu().numpy()
    # the step's min-max micro-units vs the oracle's normalize_scores + "%.6f"
    o_norm = coracle.minmax_per_query(h["raw"], h["off"])
    o_micro = np.array([int(f"{v:.6f}".replace(".", "")) for v in o_norm], np.int64)
    ok = bool(np.array_equal(h["micro"].astype(np.int64), o_micro))
    for m, name in enumerate(p.methods):
        if name not in METHODS:  # learned fusion: checked by tests/test_gpu_learned.py
            continue
        _, o_uc, o_perm, o_fused = coracle.fuse(h["off"], h["docid"], sc, p.R, name, 60,
                                                weights=h["w"])
        f = p.out.fused[m, : nq * p.R * p.K].cpu().numpy()  # by first-seen index u
        pm = p.out.perm[m, : nq * p.R * p.K].cpu().numpy().view(np.uint16)
        ok &= bool(np.array_equal(uc, o_uc))
        for q in range(nq):
            b, n = h["off"][q * p.R], uc[q]
            ranked = f[b + pm[b:b + n].astype(np.int64)]  # rank order, as the oracle's
            ok &= ranked.tobytes() == o_fused[b:b + n].tobytes()
            ok &= bool(np.array_equal(pm[b:b + n], o_perm[b:b + n]))
    return ok


# queries per CPU-baseline process (16 processes at most): C2's 125 make SURVEY §8(d)'s
# 2,000-query sample (~40 s wall on 16 cores; per_core_value is its single-core rate)
CPU_SAMPLE_PER_WORKER = {"c1": 1000, "c2": 125, "c3": 60, "c4": 60, "c5": 25}


def _port_frames(h, R, names, q0, qids):
    """Host sample -> the reference's {ranker: DataFrame} (rows in file order)."""
    import pandas as pd
    frames, raw_lists = {}, {}
    for r, name in enumerate(names):
        rows_q, rows_d, rows_r, rows_s = [], [], [], []
        for q in range(len(qids)):
            a, b = h["off"][(q0 + q) * R + r], h["off"][(q0 + q) * R + r + 1]
            rows_q += [qids[q]] * (b - a)
            rows_d += [f"doc{d}" for d in h["docid"][a:b]]
            rows_r += list(range(1, b - a + 1))
            rows_s += (h["micro"][a:b] / 1e6).tolist()
            raw_lists[(qids[q], name)] = h["raw"][a:b].tolist()
        frames[name] = pd.DataFrame({"qid": rows_q, "iter": "Q0", "docno": rows_d,
                                     "rank": rows_r, "score": rows_s, "runid": name})
    return frames, raw_lists


def _cpu_worker(job):
    """One CPU-baseline worker: its slice of the sample through oracle/ref_port.py —
    the reference's per-row algorithm (QPPBridge restated, pandas groupby/iterrows,
    ranx-equivalent dict loops) — timed per stage, single-threaded."""
    os.environ["OMP_NUM_THREADS"] = "1"
    from oracle import ref_port
    h, R, names, q0, nq, q_begin, methods, qpp_on, qpp_index = job
    qids = [f"test{q_begin + q0 + q}" for q in range(nq)]
    frames, raw_lists = _port_frames(h, R, names, q0, qids)
    t = {}
    t0 = time.perf_counter()
    qpp = {q: {n: [0.5] * 13 for n in names} for q in qids}
    if qpp_on:  # per (query, retriever) list, Java restated in Python (QPPBridge.java:134-453)
        for i, qid in enumerate(qids):
            for name in names:
                d = ref_port.java_qpp(int(h["nt"][q0 + i]), float(h["tf"][q0 + i][0]),
                                      float(h["tf"][q0 + i][1]),
                                      sorted(raw_lists[(qid, name)], reverse=True)[:100])
                qpp[qid][name] = [d[n] for n in ref_port.QPP_NAMES]
    t["qpp"] = time.perf_counter() - t0
    for m in methods:
        t1 = time.perf_counter()
        if m == "learned":  # src/fusion.py:387-448: .qpp round trip, GBDT, weighted groupby-sum
            from oracle import lgbm_oracle
            from qppfuse import lgbm
            model = lgbm.load_fusion_model(ROOT / "tests" / "golden" / "lgbm" /
                                           "nq_fusion_multioutput.json.gz")
            norm = {}
            for name in names:  # per .qpp file: min-max over its queries, "%.6f" text
                col = ref_port.normalize_qpp({q: qpp[q][name] for q in qids}, "minmax")
                for q in qids:
                    norm.setdefault(q, {})[name] = [float(f"{x:.6f}") for x in col[q]]
            wd = lgbm_oracle.weights_dict(frames, norm, model)
            ref_port.learned_fusion_from_weights(frames, wd, len(model.retrievers))
        else:
            ref_port.fuse(frames, m, qpp, qpp_index, 60)
        t[m] = time.perf_counter() - t1
    rows = int(sum(len(df) for df in frames.values()))
    return nq, time.perf_counter() - t0, t, rows


def cpu_baseline_port(p: Pipeline, per_worker: int, workers: int):
    """The reference's CPU path on a bounded sample: `workers` processes, each timing
    `per_worker` queries single-threaded; value = sample / slowest worker's time."""
    import multiprocessing as mp
    nq = min(per_worker * workers, p.Q)
    workers = max(1, min(workers, nq))
    h = host_sample(p, nq)
    bounds = [nq * i // workers for i in range(workers + 1)]
    jobs = []
    for i in range(workers):
        a, b = bounds[i], bounds[i + 1]
        sub = dict(off=h["off"], docid=h["docid"], raw=h["raw"], micro=h["micro"],
                   nt=h["nt"], tf=h["tf"])
        jobs.append((sub, p.R, NAMES[:p.R], a, b - a, p.q_begin, p.methods, p.args.wl["qpp"],
                     p.args.qpp_index))
    t0 = time.perf_counter()
    with mp.get_context("spawn").Pool(workers) as pool:
        res = pool.map(_cpu_worker, jobs)
    wall = time.perf_counter() - t0
    slowest = max(r[1] for r in res)
    busy = sum(r[1] for r in res)
    stage = {k: sum(r[2][k] for r in res) for k in res[0][2]}
    rows = sum(r[3] for r in res)
    out = {"value": round(nq / slowest, 4), "per_core_value": round(nq / busy, 4),
           "sample_queries": nq, "workers": workers, "wall_s": round(wall, 2),
           "stage_s_all_workers": {k: round(v, 2) for k, v in stage.items()}}
    if "wcombsum" in stage:  # calibration: the survey timed the reference itself at
        out["wcombsum_us_per_row"] = round(stage["wcombsum"] / rows * 1e6, 2)  # 30.8 us/row
    return out


def cpu_baseline_native(p: Pipeline, nq: int):
    from oracle import _loader as coracle
    h = host_sample(p, nq)
    sc = h["micro"].astype(np.float64) / 1e6
    t0 = time.perf_counter()
    for m in p.methods:
        # learned fusion's native cost: the same weighted per-document sum (the C
        # oracle has no Kahan / docid-tie variant; the loop shape is W-CombSUM's)
        coracle.fuse(h["off"], h["docid"], sc, p.R, "wcombsum" if m == "learned" else m, 60,
                     weights=h["w"])
    coracle.qpp_raw(h["raw"], h["off"], np.repeat(h["nt"], p.R), np.repeat(h["tf"][:, 0], p.R),
                    np.repeat(h["tf"][:, 1], p.R))
    dt = time.perf_counter() - t0
    return nq / dt


def cpu_calibration():
    """The newest committed tools/calibrate_cpu.py result: reference / port time ratio
    of weighted_combsum / weighted_rrf, measured side by side on the build host."""
    files = sorted((ROOT / "profiles").glob("r*_cpu_calibration.json"))
    if not files:
        return None
    d = json.loads(files[-1].read_text())
    return {"ratio": d["ratio"], "ratio_reference_over_port": d["ratio_reference_over_port"],
            "reference_us_per_row": d["reference_us_per_row"],
            "port_us_per_row": d["port_us_per_row"], "host": d["host"],
            "source": f"profiles/{files[-1].name} (tools/calibrate_cpu.py)"}


VALU_PEAK_PER_SIMD_NS = 0.5208  # tools/valu_peak.hip on MI355X (profiles/r01_valu.json)
N_SIMDS = 1024


def pmc_valu(args, kernel_substr="qf_fuse (sum of its kernels)"):
    """VALU instructions per qf_fuse launch (SQ_INSTS_VALU) from the committed summary."""
    default = args.workload == "c2" and args.queries in (None, 3452) and \
        (args.retrievers, args.k) == (5, 1000)
    files = sorted((ROOT / "profiles").glob("r*_pmc.json"))
    if not default or not files:
        return None
    for name, d in json.loads(files[-1].read_text()).items():
        if kernel_substr in name and d.get("insts_valu"):
            return d["insts_valu"]
    return None


def pmc_traffic(args, kernel_substr="qf_fuse (sum of its kernels)"):
    """HBM bytes per qf_fuse launch from the newest committed rocprofv3 PMC summary.

    profiles/rNN_pmc.json is produced by tools/profile.sh + tools/summarize_profile.py
    from FETCH_SIZE and WRITE_SIZE passes (separate runs) of this same bench command
    at its default workload; it only applies to that workload.
    """
    default = args.workload == "c2" and args.queries in (None, 3452) and \
        (args.retrievers, args.k) == (5, 1000)
    files = sorted((ROOT / "profiles").glob("r*_pmc.json"))
    if not default or not files:
        return None, None
    data = json.loads(files[-1].read_text())
    for name, d in data.items():
        if kernel_substr in name and d.get("hbm_bytes"):
            if "fetch_calibration" not in data:  # an old summary: FETCH_SIZE uncorrected
                return d["hbm_bytes"], f"{files[-1].name}: FETCH_SIZE+WRITE_SIZE x1024"
            return d["hbm_bytes"], (f"{files[-1].name}: (FETCH_SIZE x2 + WRITE_SIZE) x1024 "
                                    f"(gfx950 FETCH correction, checked on the min-max kernel)")
    return None, None


def timed_loop(p: Pipeline, steps: int, world: int, dev) -> float:
    """Barrier + synchronize, `steps` steps, synchronize + barrier; max over ranks."""
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        p.step(timed=True)
    p.drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def copy_ceiling_gbs(dev, nbytes: int = 1 << 30, reps: int = 40) -> dict:
    """Measured device-to-device copy rates (read + write bytes / s): the practical HBM
    ceiling next to the 8 TB/s spec peak.  `kernel`: the library's
    hand-written 16-byte-per-lane streaming copy (qf_stream_copy, csrc/qf_norm.hip) —
    the ceiling; `blit`: torch's copy_ (the runtime's copyBuffer blit), for the record."""
    from qppfuse import _lib
    a = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    a.fill_(1.0)
    s = torch.cuda.current_stream().cuda_stream
    kcopy = lambda: _lib.call("qf_stream_copy", b.data_ptr(), a.data_ptr(), nbytes, s)
    out = {}
    for name, fn in (("kernel", kcopy), ("blit", lambda: b.copy_(a))):
        for _ in range(4):  # the first copies run while the clocks ramp
            fn()
        # the best of `blocks` back-to-back blocks of reps / blocks copies: a ceiling
        blocks, best = 4, float("inf")
        for _ in range(blocks):
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            for _ in range(reps // blocks):
                fn()
            s1.record()
            torch.cuda.synchronize()
            best = min(best, s0.elapsed_time(s1) / (reps // blocks))
        out[name] = 2 * nbytes / (best * 1e-3) / 1e9
    del a, b
    return out


def progress(msg: str):
    """One line on stderr per phase (long runs are not silent; stdout stays one JSON line)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    # stdout carries exactly one JSON line: everything else (library banners such as
    # gloo's, progress) goes to stderr; the result is written on the saved stdout
    out_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    world, rank, dev = setup_dist(args)
    if args.gather_topk is None:
        args.gather_topk = 100 if world > 1 else 0
    from qppfuse import _lib
    _lib.lib()
    progress(f"rank {rank}/{world}: generating {args.workload} inputs")
    p = Pipeline(args, world, rank, dev)
    progress(f"rank {rank}: {p.Q} queries x {p.R} x top-{p.K} resident; warmup {args.warmup}")
    # the device-copy ceiling of the roofline object, measured before the warmup steps:
    # ~10 ms of HBM traffic that also takes the GPU out of its idle clocks, so a short
    # timed region (the driver's 5 + 20 steps) sees the steady-state step time
    copy = copy_ceiling_gbs(dev)
    copy_gbs = copy["kernel"]
    for _ in range(args.warmup):
        p.step()
    p.drain()
    p.wait_s, p.timed_steps = 0.0, 0
    progress(f"rank {rank}: timing {args.steps} steps")
    elapsed = timed_loop(p, args.steps, world, dev)
    total_q = p.Q * args.steps
    if world > 1:
        import torch.distributed as dist
        qt = torch.tensor([p.Q], dtype=torch.int64, device=dev)
        dist.all_reduce(qt)
        total_q = int(qt.item()) * args.steps
    without_gather = None
    if world > 1 and args.gather_topk > 0:  # the same step without the collective
        k, args.gather_topk = args.gather_topk, 0
        ms_fuse = list(p.ev)
        e2 = timed_loop(p, args.steps, world, dev)
        p.ev, args.gather_topk = ms_fuse, k
        without_gather = {"value": round(total_q / e2, 2),
                          "ms_per_step": round(e2 / args.steps * 1e3, 4)}
    gather_info = None
    if p.gather is not None:
        into0 = (p.world - 1) * p.gather.nbytes  # the peers' buffers (rank 0's own stays local)
        step_s = elapsed / args.steps
        gather_info = {
            "topk": args.gather_topk, "bytes_per_rank_per_step": p.gather.nbytes,
            "bytes_into_rank0_per_step": into0,
            "ingress_gbs_at_measured_step": round(into0 / step_s / 1e9, 2),
            "rank0_host_wait_ms_per_step": round(p.wait_s / max(1, p.timed_steps) * 1e3, 4),
            "step_ms_without_gather": None if without_gather is None
            else without_gather["ms_per_step"],
            "gather_cost_ms_per_step": None if without_gather is None
            else round(step_s * 1e3 - without_gather["ms_per_step"], 4),
            "note": "RCCL wait() only orders the compute stream behind the gather (no host "
                    "block), so the host wait is ~0 there; the gather's cost on the step is "
                    "ms_per_step - step_ms_without_gather (DESIGN.md §7's ingress budget)"}
    value = total_q / elapsed
    fuse_ms = p.fuse_kernel_ms()
    fbytes, mean_u = p.fuse_bytes()
    achieved = fbytes / (fuse_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(args)
    valu = pmc_valu(args)
    progress(f"rank {rank}: {elapsed / args.steps * 1e3:.3f} ms/step; parity + NDCG checks")
    parity = check_parity(p, min(args.check, p.Q)) if args.check > 0 else None
    gparity = p.gather_parity()
    ndcg_vals, eval_ms = ndcg_device(p)
    result = None
    if rank == 0:
        cpu = None
        ported = all(m in METHODS or m == "learned" for m in p.methods)
        per_worker = (CPU_SAMPLE_PER_WORKER[args.workload] if args.cpu_sample is None
                      else args.cpu_sample)
        if world == 1 and per_worker > 0 and ported:
            workers = args.cpu_workers or min(16, os.cpu_count() or 1)
            progress(f"CPU baseline: {workers} processes x {per_worker} queries")
            c = cpu_baseline_port(p, per_worker, workers)
            cpu = {"value": c["value"], "unit": "fused queries/s", "cores": c["workers"],
                   "kind": "port",
                   # "state nproc" — the host's CPUs and this process's share
                   "host_nproc": os.cpu_count(),
                   "host_cpus_allowed": len(os.sched_getaffinity(0)),
                   "sample": f"{c['sample_queries']} queries x {args.retrievers} x top-{args.k}"
                             f"{' + 13 QPP predictors' if args.wl['qpp'] else ''} + "
                             f"{len(p.methods)} fusion(s) through oracle/ref_port.py (the "
                             f"reference's per-row algorithm: pandas groupby/iterrows, "
                             f"ranx-equivalent dict loops), {c['workers']} single-threaded "
                             f"processes, {c['wall_s']} s wall",
                   **{k: v for k, v in c.items() if k not in ("value", "workers")}}
            cal = cpu_calibration()
            if cal is not None:  # the port vs the reference itself, timed on one host
                cpu["calibration"] = cal
                cpu["reference_equivalent_value"] = round(c["value"] / cal["ratio"], 4)
            if args.native_sample > 0:
                cpu["native_c_oracle_value"] = round(
                    cpu_baseline_native(p, min(args.native_sample, p.Q)), 2)
        result = {
            "metric": "fused queries/sec (5 retrievers x top-1000), all 6 fusions + 13 QPP"
                      if args.workload == "c2" else
                      f"fused queries/sec ({args.retrievers} retrievers x top-{args.k}), "
                      f"{args.workload.upper()}",
            "value": round(value, 2), "unit": "fused queries/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "strong" if args.wl["total"] and args.queries is None else "weak",
            "vs_baseline": None, "dtype": "f64",
            "data": ("synthetic: SURVEY.md §8(d) generator (qf_synth_runs_nq, DESIGN.md §4.5): "
                     "per list 1000 distinct ids, p 0.5 from a 2K shared pool else the 2,681,468 "
                     "NQ ids; BM25/Splade Gamma(2,6)+5, BGE/BM25_TCT 0.5+0.4 Beta(5,2), "
                     "BM25_MonoT5 ln Beta(5,2), sorted + 1e-6 tie-breaker; the real NQ test "
                     "qrels (4,201) planted at Geometric(0.15) ranks, p_r 0.9/0.5/0.9/0.8/0.9"
                     if args.generator == "nq" else
                     "synthetic (rounds 1-4 exp-decay generator, qf_synth_runs)"),
            "config": {"workload": args.wl["desc"],
                       "queries_per_gpu": p.Q, "retrievers": args.retrievers,
                       "k": args.k, "qpp_top_k": args.qpp_top_k, "methods": p.methods,
                       "parallelism": f"query-sharded x{world}", "mean_union": round(mean_u, 1),
                       "sharding": ("contiguous query ranges balanced by the entry count "
                                    "(qppfuse.dist.shard_by_entries over the run set's list "
                                    "offsets): shard sizes " + str(p.shard_sizes)
                                    if p.plan is not None else
                                    f"weak scaling: {p.Q} queries per rank, rank r at r x {p.Q}"),
                       "generator": args.generator,
                       "gather_topk_to_rank0": args.gather_topk,
                       "qids": (None if p.qids is None else
                                f"real BEIR test qids, namespaced: {p.qids[0]} .. {p.qids[-1]}"),
                       "without_gather": without_gather, "gather": gather_info},
            "roofline": {"bound": "hbm", "kernel": "qf_fuse", "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": fbytes,
                         "kernel_ms": round(fuse_ms, 4),
                         # the roof it actually meets: VALU issue
                         "valu_issue_frac": None if valu is None else round(
                             valu / N_SIMDS / (fuse_ms * 1e6) / VALU_PEAK_PER_SIMD_NS, 4),
                         "valu_insts_per_launch": valu,
                         "copy_ceiling_gbs": round(copy_gbs, 1),
                         "copy_ceiling_source": "qf_stream_copy: 16 B/lane non-temporal "
                                                "copy, one access per thread, one-shot grid, "
                                                "1 GiB, read + write, best of 4 x 10",
                         "copy_blit_gbs": round(copy["blit"], 1),
                         "frac_of_copy_ceiling": round(achieved / copy_gbs, 4)},
            "cpu_baseline": cpu,
            "parity_vs_oracle": {"queries": min(args.check, p.Q), "bit_exact": parity},
            "gather_parity": gparity,
            "ndcg10": {m: round(float(np.nanmean(ndcg_vals[i])), 6)
                       for i, m in enumerate(p.methods)},
            "ndcg10_eval_ms": round(eval_ms, 4),
        }
        if world == 1 and args.ndcg_sample > 0 and all(m in METHODS for m in p.methods):
            nq = min(args.ndcg_sample, p.Q)
            dq, dm = ndcg_delta(p, ndcg_vals, nq)
            result["ndcg10_delta_vs_ref"] = {
                "queries": nq, "max_abs_per_query": dq, "max_abs_mean": dm,
                "ref": "CPU reference path: C oracle fusion + trec_eval restatement "
                       "(oracle/), scores as the .res text"}
        elif world == 1 and args.ndcg_sample > 0 and p.methods == ["learned"]:
            nq = min(args.ndcg_sample, p.Q)
            dq, dm = ndcg_delta_learned(p, ndcg_vals, nq)
            result["ndcg10_delta_vs_ref"] = {
                "queries": nq, "max_abs_per_query": dq, "max_abs_mean": dm,
                "ref": "CPU reference path: QPP by the Java restatement (oracle/qpp_oracle.c), "
                       "min-max + '%.6f', LightGBM walk restated (oracle/lgbm_oracle.py), "
                       "pandas' Kahan groupby-sum in run order, trec_eval restatement"}
        os.write(out_fd, (json.dumps(result) + "\n").encode())
    if world > 1:
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
