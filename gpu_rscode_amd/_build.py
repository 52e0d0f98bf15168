"""In-tree native build driver (``make -C csrc``).

Artifacts are built next to the sources so they travel with the repository snapshot to the GPU
box: ``gpu_rscode_amd/_hip.so`` (gfx950 kernels + runtime), ``gpu_rscode_amd/_cpu.so`` (CPU codec),
``bin/RS`` and ``bin/CPU-RS`` (CLIs), ``lib/libgfrs.so`` (the C API, ``csrc/include/gfrs.h``) and
``bin/gfrs_capi_demo``. ``make`` is incremental, so calling :func:`build` when
everything is up to date costs a few milliseconds.
"""
from __future__ import annotations

import contextlib
import fcntl
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
    # make left these current with respect to their own dependencies; stamp them so that a source
    # they do not depend on (a kernel edit for _cpu.so) does not mark them stale to the loader
    for p in TARGET_OUTPUTS.get(target, ()):
        if p.exists():
            os.utime(p)
    if not quiet:
        print(res.stdout)


@contextlib.contextmanager
def file_lock(shared: bool = False):
    """Lock across processes (``flock`` on ``build/.lock``): ranks started together by torchrun
    serialise their rebuilds (exclusive) instead of overwriting one module concurrently, and check
    staleness and import under the shared lock, so no rank reads a module while another links it."""
    path = ROOT / "build" / ".lock"
    path.parent.mkdir(parents=True, exist_ok=True)
    with open(path, "a") as f:
        fcntl.flock(f, fcntl.LOCK_SH if shared else fcntl.LOCK_EX)
        try:
            yield
        finally:
            fcntl.flock(f, fcntl.LOCK_UN)


def have_sources() -> bool:
    """False for an installed copy of the package (``pip install``): no ``csrc/`` next to it, the
    modules were built at install time and are used as they are."""
    return (CSRC / "Makefile").exists()


SOURCE_SUFFIXES = (".hip", ".cpp", ".h", ".hpp")
_HIP_OUT = (PKG / "_hip.so", ROOT / "bin" / "RS")
_CPU_OUT = (PKG / "_cpu.so", ROOT / "bin" / "CPU-RS")
TARGET_OUTPUTS = {"hip": _HIP_OUT, "cpu": _CPU_OUT, "all": _HIP_OUT + _CPU_OUT}


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
