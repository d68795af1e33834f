"""cProfile of load_runs on C2-shaped files (development tool; e2e.py's generator)."""
import cProfile
import pstats
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tools"), str(ROOT / "qpp-fusion-rag_amd")]
import e2e  # noqa: E402
from qppfuse import fusion  # noqa: E402

d = Path(tempfile.mkdtemp(prefix="qf_prof_"))
e2e.generate(d, 3452, 5, 1000)
for _ in range(2):
    fusion._PACK_CACHE.clear()
    t = time.perf_counter()
    runs = fusion.load_runs(str(d))
    print("load_runs", round(time.perf_counter() - t, 4), flush=True)
    del runs
fusion._PACK_CACHE.clear()
cProfile.run("runs = fusion.load_runs(str(d))", "/tmp/qf_load.prof")
pstats.Stats("/tmp/qf_load.prof").sort_stats("tottime").print_stats(25)
