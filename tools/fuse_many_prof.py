"""Where fuse_many's time goes on C2-shaped files (development): the pack-cache
check, the QPP weights, the upload, the kernels, the copy back.
python tools/fuse_many_prof.py [--dir DIR]   (files made by tools/e2e.py's generator)"""
import argparse
import json
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "qpp-fusion-rag_amd"), str(ROOT / "tools")]
import torch  # noqa: E402

METHODS = ["combsum", "combmnz", "rrf", "wcombsum", "wcombmnz", "wrrf"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default=None)
    a = ap.parse_args()
    from qppfuse import fusion
    import e2e
    d = Path(a.dir or tempfile.mkdtemp(prefix="qf_fmp_"))
    torch.cuda.set_device(0)
    if not any(d.glob("*.norm.res")):
        e2e.generate(d, 3452, 5, 1000)
    runs = fusion.load_runs(str(d))
    qpp = fusion.load_qpp_scores(str(d / "qpp"))
    T = {}

    def timed(name, fn):
        def w(*args, **kw):
            torch.cuda.synchronize()
            t = time.perf_counter()
            r = fn(*args, **kw)
            torch.cuda.synchronize()
            T[name] = T.get(name, 0.0) + time.perf_counter() - t
            return r
        return w

    fusion._pack = timed("pack (cache check)", fusion._pack)
    fusion._weights = timed("qpp weights", fusion._weights)
    orig_to_device = fusion.RunSet.to_device
    fusion.RunSet.to_device = timed("upload", orig_to_device)
    fusion.engine.fuse = timed("kernels", fusion.engine.fuse)
    for rep in range(4):
        T.clear()
        rs = fusion._PACK_CACHE and next(iter(fusion._PACK_CACHE.values()))[1]
        if rs:
            rs._device = None  # upload again each repeat
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fusion.fuse_many(runs, METHODS, qpp, 5)
        torch.cuda.synchronize()
        tot = time.perf_counter() - t0
        rest = tot - sum(T.values())
        print(json.dumps({"total_s": round(tot, 4), **{k: round(v, 4) for k, v in T.items()},
                          "copy back + FusedRun": round(rest, 4)}), flush=True)
        time.sleep(0.5)  # let the background pinning of the first call finish


if __name__ == "__main__":
    main()
