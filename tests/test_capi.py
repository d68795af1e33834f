"""The C-ABI library loads and exports every symbol include/qppfuse.h declares (CPU)."""
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "qppfuse.h"


def header_functions():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(qf_\w+)\s*\(", text, re.M)))


def test_header_declares_expected_entry_points():
    fns = header_functions()
    for name in ["qf_fuse", "qf_minmax_per_query", "qf_qpp_raw", "qf_qpp_colminmax",
                 "qf_qpp_normalize", "qf_last_error", "qf_version", "qf_max_entries_per_query",
                 "qf_synth_runs", "qf_eval", "qf_gbdt_predict", "qf_learned_weights",
                 "qf_qpp_colmeanstd", "qf_fuse_probfuse", "qf_qpp_features"]:
        assert name in fns


def test_library_exports_every_declared_symbol():
    from qppfuse import _lib
    lib = _lib.lib()
    for name in header_functions():
        assert hasattr(lib, name), name
        assert name in _lib.SIGNATURES, f"{name} has no ctypes signature"
    assert set(_lib.SIGNATURES) == set(header_functions())


def test_io_library_exports_every_declared_symbol():
    """libqfio.so (host run-file I/O) exports every qfio_ function include/qfio.h
    declares, and qppfuse.fastio binds each with a ctypes signature."""
    import ctypes
    from qppfuse import fastio
    text = (ROOT / "include" / "qfio.h").read_text()
    names = sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(qfio_\w+)\s*\(", text, re.M)))
    assert {"qfio_load_runs", "qfio_write_run", "qfio_gather_strings", "qfio_gather_chars",
            "qfio_repeat_offsets", "qfio_hash_bytes"} <= set(names)
    lib = fastio.lib()
    for name in names:
        fn = getattr(lib, name)
        assert isinstance(fn, ctypes._CFuncPtr), name
        assert fn.argtypes is not None or name in ("qfio_last_error",), f"{name} is not bound"


def test_version_and_limits():
    from qppfuse import _lib
    assert "gfx950" in _lib.version()
    # LDS kernels to 10,240 entries, the workspace kernel beyond; perm / u are uint16
    assert _lib.max_entries_per_query() == 65535


def test_argument_validation_without_device():
    """Validation happens before any HIP call: bad arguments fail with EINVAL."""
    from qppfuse import _lib
    tail = (None, None, None, None, 0, None)
    with pytest.raises(ValueError, match="n_retrievers"):
        _lib.call("qf_fuse", 1, 0, None, None, None, 0, None, None, 1, 60, 10, *tail)
    with pytest.raises(ValueError, match="method mask"):
        _lib.call("qf_fuse", 1, 2, None, None, None, 0, None, None, 0x200, 60, 10, *tail)
    with pytest.raises(ValueError, match="segment table"):
        _lib.call("qf_fuse", 1, 2, None, None, None, 0, None, None, _lib.PROBFUSE, 60, 10, *tail)
    with pytest.raises(ValueError, match="segment table"):
        _lib.call("qf_fuse_probfuse", 1, 2, None, None, None, 0, None, None, _lib.PROBFUSE, 60,
                  None, 25, 100, 10, *tail)
    with pytest.raises(ValueError, match="without weights"):
        _lib.call("qf_fuse", 1, 2, None, None, None, 0, None, None, _lib.WRRF_MUL, 60, 10, *tail)
    with pytest.raises(ValueError, match="different weights"):
        _lib.call("qf_fuse", 1, 2, None, None, None, 0, None, 8, _lib.LEARNED | _lib.WRRF, 60, 10,
                  *tail)
    with pytest.raises(ValueError, match="without weights"):
        _lib.call("qf_fuse", 1, 2, None, None, None, 0, None, None, _lib.WRRF, 60, 10, *tail)
    with pytest.raises(_lib.QPPFuseError, match="exceed"):
        _lib.call("qf_fuse", 1, 2, None, None, None, 0, None, None, _lib.RRF, 60, 10**6, *tail)
    with pytest.raises(ValueError, match="null buffer"):
        _lib.call("qf_fuse", 1, 2, 8, 8, 8, 0, None, None, _lib.RRF, 60, 10, 8, 8, 8, None, 16,
                  None)
    import ctypes as C
    import numpy as np
    kind = np.array([0], np.int32)
    cut = np.array([0], np.int32)
    with pytest.raises(ValueError, match="cutoff"):
        _lib.call("qf_eval", 1, 8, 1, None, 8, None, 8, 0, 1, 0, 8, 8, 8, 1, 1,
                  kind.ctypes.data, cut.ctypes.data, 8, None)
    cut[0] = 10
    with pytest.raises(_lib.QPPFuseError, match="judged"):
        _lib.call("qf_eval", 1, 8, 1, None, 8, None, 8, 0, 1, 0, 8, 8, 8, 10**6, 1,
                  kind.ctypes.data, cut.ctypes.data, 8, None)
    with pytest.raises(ValueError, match="null buffer"):
        _lib.call("qf_eval", 1, None, 1, None, 8, None, 8, 0, 1, 0, 8, 8, 8, 1, 1,
                  kind.ctypes.data, cut.ctypes.data, 8, None)
    with pytest.raises(ValueError, match="qpp_index"):
        _lib.call("qf_qpp_normalize", 1, 1, 1, 1, 1, 1, 13, None, None, None, None)
    # qf_fuse_qpp's QPP-weight arguments (checked before any device work)
    W, L = 1 << 3, 1 << 6  # QF_WCOMBSUM, QF_LEARNED
    fq = lambda raw, stats, mode, idx, methods: (2, 3, 8, 8, 8, 1, None, raw, stats, mode, idx,
                                                methods, 60, 10, 8, 8, 8, 8, 10, None)
    with pytest.raises(ValueError, match="QPP weight"):
        _lib.call("qf_fuse_qpp", *fq(8, 8, 1, 13, W))
    with pytest.raises(ValueError, match="QPP weight"):
        _lib.call("qf_fuse_qpp", *fq(8, None, 1, 5, W))   # min-max needs the statistics
    with pytest.raises(ValueError, match="QPP weight"):
        _lib.call("qf_fuse_qpp", *fq(8, 8, 7, 5, W))
    with pytest.raises(ValueError, match="learned"):
        _lib.call("qf_fuse_qpp", *fq(8, 8, 1, 5, L))
    with pytest.raises(ValueError, match="null buffer"):
        _lib.call("qf_fuse_qpp", *fq(None, 8, 1, 5, W))
    # the one-launch learned weights: host-side size and map checks (no device needed)
    blocks = np.array([0, 1, -1], np.int32)
    rb = np.array([0, 1, -1], np.int32)
    args = lambda nb, nboost, rbp, rblk: (5, 8, None, None, None, 0, 3, rblk.ctypes.data, nb,
                                         nboost, 8, 8, 8, 8, 8, 8, 8, 8, 8, 3, rbp.ctypes.data,
                                         None, 8, None)
    with pytest.raises(ValueError, match="bad sizes"):
        _lib.call("qf_learned_gbdt_weights", *args(20, 3, rb, blocks))  # 20 x 13 > 256 features
    with pytest.raises(ValueError, match="bad sizes"):
        _lib.call("qf_learned_gbdt_weights", *args(3, 17, rb, blocks))  # boosters > 16
    with pytest.raises(ValueError, match="run_of_block"):
        _lib.call("qf_learned_gbdt_weights", *args(3, 3, rb, np.array([0, 3, 1], np.int32)))
    with pytest.raises(ValueError, match="run_to_booster"):
        _lib.call("qf_learned_gbdt_weights", *args(3, 3, np.array([0, 3, 1], np.int32), blocks))
    with pytest.raises(ValueError, match="null buffer"):
        _lib.call("qf_learned_gbdt_weights", 5, None, 8, None, None, 1, 3, blocks.ctypes.data, 3,
                  3, 8, 8, 8, 8, 8, 8, 8, 8, 8, 3, rb.ctypes.data, None, 8, None)


def test_product_has_no_cpu_fallback(monkeypatch):
    """Without a device the product raises instead of computing on the CPU."""
    import torch
    from qppfuse import engine
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        engine.require_device()


def test_product_never_imports_oracle():
    pkg = ROOT / "qpp-fusion-rag_amd"
    for f in pkg.rglob("*.py"):
        assert "oracle" not in re.findall(r"^\s*(?:from|import)\s+(\w+)", f.read_text(), re.M), f


def test_package_reexports_reference_names():
    """src/__init__.py:28,37 re-exports these; qppfuse does too, lazily."""
    import subprocess
    import sys
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "import qppfuse\n"
        "from qppfuse import _lib\n"
        "assert _lib._LIB is None, 'importing the package loaded the library'\n"
        "assert 'qppfuse.fusion' not in sys.modules and 'torch' not in sys.modules\n"
        "from qppfuse import (QPPBridge, compute_qpp_for_res_file, combsum, combmnz, rrf,\n"
        "                     weighted_combsum, weighted_rrf, learned_fusion)\n"
        "import qppfuse.fusion as F, qppfuse.qpp as Q\n"
        "assert combsum is F.combsum and weighted_rrf is F.weighted_rrf\n"
        "assert learned_fusion is F.learned_fusion and QPPBridge is Q.QPPBridge\n"
        "assert compute_qpp_for_res_file is Q.compute_qpp_for_res_file\n"
        "assert _lib._LIB is None\n"
        "print('ok')\n") % str(ROOT / "qpp-fusion-rag_amd")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr[-2000:]
    import qppfuse
    with pytest.raises(AttributeError):
        qppfuse.no_such_name  # noqa: B018


def test_stream_copy_validation():
    from qppfuse import _lib
    with pytest.raises(ValueError, match="16-byte"):
        _lib.call("qf_stream_copy", 16, 16, 8, None)
    with pytest.raises(ValueError, match="16-byte"):
        _lib.call("qf_stream_copy", 17, 16, 16, None)
    _lib.call("qf_stream_copy", None, None, 0, None)  # nothing to copy: no HIP call


def test_fuse_workspace_bytes():
    """qf_fuse_workspace_bytes is host arithmetic: 0 without the workspace kernel,
    the stream-ordered allocation's size with it (capped at 4 GB, two workgroups
    per CU at most)."""
    from qppfuse import engine
    assert engine.workspace_bytes(3452, 5, 5000, ["combsum"]) == 0
    assert engine.workspace_bytes(3452, 10, 10240, ["combsum"]) == 0
    one = engine.workspace_bytes(1, 5, 100_000, ["combsum"])
    two = engine.workspace_bytes(2, 5, 100_000, ["combsum"])
    assert one > 0 and two == 2 * one
    assert engine.workspace_bytes(10**6, 5, 100_000, ["rrf"]) <= 4 << 30
    assert engine.workspace_bytes(4, 20, 500, ["rrf"]) > 0   # > 16 runs: the workspace kernel
    assert engine.workspace_bytes(0, 5, 100_000, ["rrf"]) == 0


def test_fuse_ws_rejects_a_short_workspace():
    from qppfuse import _lib, engine
    need = engine.workspace_bytes(1, 5, 100_000, ["rrf"])
    with pytest.raises(ValueError, match="workspace"):
        _lib.call("qf_fuse_ws", 1, 5, 8, 8, 8, 0, None, None, _lib.RRF, 60, 100_000, 8, 8, 8, 1,
                  8, 16, 256, need - 1, None)


def test_fuse_ws_rejects_a_misaligned_workspace():
    """Each workgroup's share of the workspace holds u32 atomicCAS targets and u64
    sort words, so the base must be 256-byte aligned: a slice such as
    ws[1:] of a torch buffer fails with EINVAL before any device work."""
    from qppfuse import _lib, engine
    need = engine.workspace_bytes(1, 5, 100_000, ["rrf"])
    for base in (8, 256 + 16, 4096 + 1):
        with pytest.raises(ValueError, match="256-byte aligned"):
            _lib.call("qf_fuse_ws", 1, 5, 8, 8, 8, 0, None, None, _lib.RRF, 60, 100_000, 8, 8, 8,
                      1, 8, 16, base, need, None)


def test_build_deps_follow_includes(tmp_path):
    """_build's dependency list comes from an #include scan of the sources, so touching
    ANY header a source includes (qf_lists.h among them) marks the library stale."""
    import os
    from qppfuse import _build
    names = {p.name for p in _build.deps(_build.SOURCES)}
    assert {"qf_lists.h", "qf_common.h", "qf_internal.h", "qf_log2_table.h", "qppfuse.h"} <= names
    assert {"qf_io.cpp", "qfio.h"} <= {p.name for p in _build.deps(_build.IO_SOURCES)}
    # a private tree: lib newer than every dependency, then one header touched
    src = tmp_path / "csrc"
    (src / "sub").mkdir(parents=True)
    (src / "a.hip").write_text('#include "h1.h"\n#include "sub/h2.h"\n')
    (src / "h1.h").write_text("#pragma once\n")
    (src / "sub" / "h2.h").write_text('#include "../h3.h"\n')
    (src / "h3.h").write_text("// leaf\n")
    lib = tmp_path / "lib.so"
    lib.write_bytes(b"")
    assert sorted(p.name for p in _build.deps(["a.hip"], src)) == ["a.hip", "h1.h", "h2.h", "h3.h"]
    for p in _build.deps(["a.hip"], src):
        os.utime(p, (1_000_000, 1_000_000))
    os.utime(lib, (2_000_000, 2_000_000))
    assert not _build._stale_against(lib, ["a.hip"], src)
    os.utime(src / "h3.h", (3_000_000, 3_000_000))  # a header two includes deep
    assert _build._stale_against(lib, ["a.hip"], src)
    # and the real library: every in-tree dependency is at most as new as the .so
    if _build.LIB_PATH.exists() and not _build._stale():
        t = _build.LIB_PATH.stat().st_mtime
        assert all(d.stat().st_mtime <= t for d in _build.deps(_build.SOURCES))
