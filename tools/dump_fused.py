"""Dump the C2 fused scores of a few queries (development: sort-window statistics)."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "qpp-fusion-rag_amd")]
import numpy as np
import torch
import bench

args = bench.parse()
args.queries = 200
args.gather_topk = 0
world, rank, dev = 1, 0, torch.device("cuda", 0)
p = bench.Pipeline(args, world, rank, dev)
p.step()
torch.cuda.synchronize()
uc = p.out.union_count.cpu().numpy()
off = p.off.cpu().numpy()
out = {"uc": uc, "off": off, "micro": p.micro.cpu().numpy(),
       "docid": p.docid.cpu().numpy(), "w": p.w.cpu().numpy()}
for m, name in enumerate(bench.METHODS):
    out[name] = p.out.ranked_fused()[m].cpu().numpy()  # rank order
    out[name + "_perm"] = p.out.perm[m].cpu().numpy()
Path("gpurun_out").mkdir(exist_ok=True)
np.savez_compressed("gpurun_out/fused_c2.npz", **out)
print("ok")
