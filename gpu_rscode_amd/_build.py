"""In-tree native build driver (``make -C csrc``).

Artifacts are built next to the sources so they travel with the repository snapshot to the GPU
box: ``gpu_rscode_amd/_hip.so`` (gfx950 kernels + runtime), ``gpu_rscode_amd/_cpu.so`` (CPU codec),
``bin/RS`` and ``bin/CPU-RS`` (CLIs), ``lib/libgfrs.so`` (the C API, ``csrc/include/gfrs.h``) and
``bin/gfrs_capi_demo``. ``make`` is incremental, so calling :func:`build` when
everything is up to date costs a few milliseconds.
"""
from __future__ import annotations

import os
import subprocess
import threading
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
PKG = Path(__file__).resolve().parent
_lock = threading.Lock()


def build(target: str = "all", jobs: int | None = None, quiet: bool = True) -> None:
    """Run ``make -C csrc <target>``. Targets: ``all``, ``hip``, ``cpu``, ``capi``."""
    jobs = jobs or min(8, os.cpu_count() or 4)
    cmd = ["make", "-C", str(CSRC), f"-j{jobs}", target]
    with _lock:
        res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"native build failed ({' '.join(cmd)}):\n{res.stdout[-4000:]}\n{res.stderr[-4000:]}")
    if not quiet:
        print(res.stdout)


def have_sources() -> bool:
    """False for an installed copy of the package (``pip install``): no ``csrc/`` next to it, the
    modules were built at install time and are used as they are."""
    return (CSRC / "Makefile").exists()


SOURCE_SUFFIXES = (".hip", ".cpp", ".h", ".hpp")


def newest_source_mtime() -> float:
    """Latest modification time over the native sources under ``csrc/`` (and its Makefile)."""
    newest = (CSRC / "Makefile").stat().st_mtime
    for p in CSRC.rglob("*"):
        if p.suffix in SOURCE_SUFFIXES:
            newest = max(newest, p.stat().st_mtime)
    return newest


def stale(path: Path) -> bool:
    """True when ``path`` is missing or older than some native source."""
    return not path.exists() or path.stat().st_mtime < newest_source_mtime()


def artifact(name: str) -> Path:
    return PKG / name


def binary(name: str) -> Path:
    return ROOT / "bin" / name
