"""Build libqppfuse.so in-tree with hipcc for gfx950.

The library is the product: qppfuse imports it with ctypes and fails loudly
when it is missing (no CPU fallback exists).  Built in-tree so the .so travels
to the GPU box with the repository snapshot.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
ROOT = PKG_DIR.parent  # qpp-fusion-rag_amd/
CSRC = ROOT / "csrc"
LIB_PATH = PKG_DIR / "libqppfuse.so"
IO_LIB_PATH = PKG_DIR / "libqfio.so"  # host run-file I/O (C++ / OpenMP)
IO_SOURCES = ["qf_io.cpp"]
SOURCES = ["qf_fuse.hip", "qf_qpp.hip", "qf_norm.hip", "qf_eval.hip", "qf_learn.hip", "qf_synth.hip",
           "qf_capi.hip"]
ARCH = os.environ.get("QPPFUSE_ARCH", "gfx950")
# -ffp-contract=off: the reference's arithmetic is sequential IEEE double; an
# FMA contraction would change bits (fusion sums, Java's Kahan sums).
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", f"--offload-arch={ARCH}"]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: install ROCm or set HIPCC")


_INCLUDE = re.compile(r'^\s*#\s*include\s*"([^"]+)"', re.M)


def deps(sources, base: Path = CSRC) -> list:
    """Every file the sources pull in through `#include "..."`, transitively (resolved
    against the including file's directory), with the sources themselves: a header
    edit must mark the library stale (a hand-kept list missed
    qf_lists.h)."""
    seen, todo = {}, [(base / s).resolve() for s in sources]
    while todo:
        f = todo.pop()
        if f in seen or not f.exists():
            continue
        seen[f] = True
        for inc in _INCLUDE.findall(f.read_text(errors="replace")):
            todo.append((f.parent / inc).resolve())
    return sorted(seen)


def _stale_against(lib: Path, sources, base: Path = CSRC) -> bool:
    if not lib.exists():
        return True
    t = lib.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps(sources, base))


def _stale() -> bool:
    return _stale_against(LIB_PATH, SOURCES)


def build_io(force: bool = False, verbose: bool = True) -> Path:
    """Compile the host I/O library qppfuse/libqfio.so (g++, OpenMP)."""
    if not force and not _stale_against(IO_LIB_PATH, IO_SOURCES):
        return IO_LIB_PATH
    cxx = os.environ.get("CXX", shutil.which("g++") or "g++")
    tmp = IO_LIB_PATH.with_suffix(".so.tmp")
    cmd = [cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-fopenmp", "-o", str(tmp)] + \
        [str(CSRC / s) for s in IO_SOURCES]
    if verbose:
        print("[qppfuse] " + " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, IO_LIB_PATH)
    return IO_LIB_PATH


def build(force: bool = False, verbose: bool = True) -> Path:
    """Compile every HIP source into qppfuse/libqppfuse.so (gfx950), and libqfio.so."""
    build_io(force, verbose)
    if not force and not _stale():
        return LIB_PATH
    cmd = [_hipcc(), *FLAGS, "-o", str(LIB_PATH)] + [str(CSRC / s) for s in SOURCES]
    if verbose:
        print("[qppfuse] " + " ".join(cmd), flush=True)
    tmp = LIB_PATH.with_suffix(".so.tmp")
    cmd[cmd.index(str(LIB_PATH))] = str(tmp)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


DEV_HOOKS = ROOT.parent / "tools" / "dev" / "qf_dev_hooks.h"


def build_variant(out: Path, extra_flags, dev: bool = False) -> Path:
    """Development builds from the same sources (A/B of -D knobs; dev=True force-includes
    tools/dev/qf_dev_hooks.h, whose QF_STOP stop points -DQF_STOP_AT=<phase> enables —
    the library itself never includes it)."""
    pre = ["-include", str(DEV_HOOKS)] if dev else []
    cmd = [_hipcc(), *FLAGS, *pre, *extra_flags, "-o", str(out)] + [str(CSRC / s) for s in SOURCES]
    subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    build(force=True)
