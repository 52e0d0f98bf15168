"""Loading of the native extension modules.

``torch`` is imported before ``_hip`` is loaded so the extension binds to the HIP runtime torch
already mapped (both carry soname ``libamdhip64.so.7``): one runtime per process, pointers and
streams interchangeable. On a machine with a GPU the HIP module is mandatory — :func:`hip` raises
instead of silently falling back to a slower path.
"""
from __future__ import annotations

import importlib
import os

import torch  # noqa: F401  (must precede the _hip import, see module docstring)

from . import _build

_mods: dict[str, object] = {}
_CLI = {"cpu": "CPU-RS", "hip": "RS"}  # the CLI each make target links beside its module


def _load(name: str, target: str):
    if name in _mods:
        return _mods[name]
    so = _build.artifact(f"_{name}.so")
    # make runs only for a module older than some source. An up-to-date module is imported as it is
    # even when make's intermediate objects are absent (a snapshot without build/): otherwise every
    # rank of a torchrun job would relink it while its peers import it. The rebuild itself holds a
    # cross-process lock and re-checks after acquiring it, so concurrent ranks build once.
    outs = (so, _build.binary(_CLI[name]))  # what make's target produces
    check = os.environ.get("GPURS_NO_BUILD") != "1" and _build.have_sources()
    if check:
        with _build.file_lock(shared=True):  # no builder is linking while we look
            need = any(map(_build.stale, outs))
        if need:
            with _build.file_lock():  # exclusive: one rank builds, the others wait and re-check
                if any(map(_build.stale, outs)):
                    try:
                        _build.build(target)
                    except (RuntimeError, OSError):
                        # a failed rebuild is only tolerable when the existing module is up to date
                        # with every source (e.g. no toolchain here); a stale .so would run old code
                        if not so.exists() or _build.stale(so):
                            raise
        with _build.file_lock(shared=True):  # (make also links to a temporary and renames it)
            mod = importlib.import_module(f"gpu_rscode_amd._{name}")
    else:
        mod = importlib.import_module(f"gpu_rscode_amd._{name}")
    _mods[name] = mod
    return mod


def cpu():
    """The C++ CPU codec module (always available; built with g++)."""
    return _load("cpu", "cpu")


def hip():
    """The gfx950 HIP module. Raises if it cannot be built or loaded."""
    return _load("hip", "hip")


def gpu_available() -> bool:
    return torch.cuda.is_available() and torch.cuda.device_count() > 0
