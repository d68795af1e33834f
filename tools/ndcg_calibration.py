"""Why the section 8(d) generator's fused NDCG@10 is high (development study, CPU only).

Plants the NQ qrels into the generator's unplanted runs (oracle/synth_oracle.c) with
per-retriever presence p_r and Geometric(g_r) ranks calibrated to the reference's own
per-ranker R@10 / R@100 on NQ (data/nq/results/figures/ranker_eval_nq.json) — the
draws independent per retriever ("indep"), shared across the retrievers ("como" 1), or
shared with probability 0.7 / 0.5 — then CombSUM / RRF by the C oracle and NDCG@10 by
the trec_eval restatement, beside each single retriever's NDCG@10 (BGE, BM25,
BM25_MonoT5, BM25_TCT, Splade).  The bench's own planting (p_r 0.9 / 0.5 /
0.9 / 0.8 / 0.9, Geometric(0.15), independent) gives CombSUM 0.883, RRF 0.991.
python tools/ndcg_calibration.py > profiles/r05_ndcg_calibration.txt
"""
import sys
import numpy as np
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tools"), str(ROOT / "qpp-fusion-rag_amd")]
from oracle import _loader as co
import bench
Q,R,K=500,5,1000
qo,qd=bench.nq_qrels()
off,doc,raw=co.synth_runs_nq(0,Q,R,K,20251212,np.zeros(1,np.int64),np.zeros(0,np.uint32))
doc=doc.copy()
names=["BGE","BM25","BM25_MonoT5","BM25_TCT","Splade"]
# reference per-ranker R@100, R@10
R100={"BGE":0.927,"BM25":0.750,"BM25_MonoT5":0.739,"BM25_TCT":0.739,"Splade":0.930}
R10={"BGE":0.723,"BM25":0.474,"BM25_MonoT5":0.669,"BM25_TCT":0.197,"Splade":0.739}
def g_for(ratio):
    lo,hi=1e-4,0.99
    for _ in range(60):
        g=(lo+hi)/2
        f=(1-(1-g)**10)/(1-(1-g)**100)
        if f<ratio: lo=g
        else: hi=g
    return g
G={n:g_for(R10[n]/R100[n]) for n in names}
P={n:R100[n]/(1-(1-G[n])**100) for n in names}
print({n:(round(P[n],3),round(G[n],4)) for n in names})
rng=np.random.default_rng(7)
def plant(mode, rho):
    d=doc.copy()
    for q in range(Q):
        rels=qd[qo[q]:qo[q+1]][:16]
        for jr,rd in enumerate(rels):
            up=rng.random(); ur=rng.random()
            taken=set()
            for r in range(R):
                n=names[r]
                u1 = up if mode=='como' else rng.random()
                u2 = ur if mode=='como' else rng.random()
                if rho<1 and mode=='como':
                    # partial correlation: mix
                    if rng.random()>rho: u1=rng.random()
                    if rng.random()>rho: u2=rng.random()
                if not (u1 < P[n]): continue
                p=int(np.floor(np.log(u2)/np.log(1-G[n])))
                if p>=K: continue
                a=off[q*R+r]; ids=d[a:a+K]
                f=np.flatnonzero(ids==rd)
                if len(f): ids[f[0]]=ids[p]
                ids[p]=rd
    return d
qrel_rel=np.ones(len(qd),np.int32)
micro=np.floor(co.minmax_per_query(raw,off)*1e6+0.5)/1e6
for mode,rho in (('indep',1),('como',1),('como',0.7),('como',0.5)):
    d=plant(mode,rho)
    out=[]
    for m in ["combsum","rrf"]:
        ud,uc,perm,fused=co.fuse(off,d,micro,R,m,60)
        roff=np.zeros(Q+1,np.int64); roff[1:]=np.cumsum(uc)
        b=off[:-1:R][:Q]
        rdoc=np.concatenate([ud[b[q]+perm[b[q]:b[q]+uc[q]].astype(np.int64)] for q in range(Q)])
        rsc=np.concatenate([fused[b[q]:b[q]+uc[q]] for q in range(Q)])
        v=co.evaluate(roff,rdoc,rsc,qo[:Q+1],qd[:qo[Q]],qrel_rel[:qo[Q]],["nDCG@10"],text=True)[:,0]
        out.append((m,round(float(np.nanmean(v)),3)))
    # single retriever ndcg
    singles=[]
    for r in range(R):
        roff=np.arange(0,Q*K+1,K); rdoc=np.concatenate([d[off[q*R+r]:off[q*R+r]+K] for q in range(Q)]); rsc=np.concatenate([raw[off[q*R+r]:off[q*R+r]+K] for q in range(Q)])
        v=co.evaluate(roff.astype(np.int64),rdoc,rsc,qo[:Q+1],qd[:qo[Q]],qrel_rel[:qo[Q]],["nDCG@10"],text=True)[:,0]
        singles.append(round(float(np.nanmean(v)),3))
    print(mode,rho,out,singles)
