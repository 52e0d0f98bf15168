"""The reference's on-disk formats, in Python.

* chunk files ``_<i>_<name>`` (``src/encode.cu:434-465``) — placed next to the input file, so
  paths with directories work (the reference breaks on them);
* ``<file>.METADATA``: ``totalSize\\n p k\\n`` then the k+p rows of ``G = [I; E]`` as ``"%d "``
  values (``src/encode.cu:61-101``); the CPU reference's 2-line form (``src/cpu-rs.c:465-476``) is
  accepted and G regenerated from the reference Vandermonde;
* decode config: whitespace-separated chunk names, row index ``atoi(basename + 1)``
  (``src/decode.cu:302-318``); ``worst_case_conf`` is ``src/unit-test.sh``.

The C++ implementation (``csrc/io/format.cpp``) is what the CLIs use; tests pin the two equal.
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass

import numpy as np

from ..gf import GF256


def chunk_path(file: str, index: int) -> str:
    d, b = os.path.split(file)
    name = f"_{index}_{b}"
    return os.path.join(d, name) if d else name


def metadata_path(file: str) -> str:
    return file + ".METADATA"


def chunk_index(name: str) -> int:
    """``atoi(basename + 1)`` of a chunk name; -1 when malformed."""
    b = os.path.basename(name)
    m = re.match(r"_(\d+)", b)
    return int(m.group(1)) if m else -1


def chunk_size(total: int, k: int) -> int:
    return max(1, (total + k - 1) // k)


@dataclass
class Metadata:
    total_size: int
    p: int
    k: int
    g: np.ndarray  # (k+p) x k
    has_matrix: bool
    crc: list | None = None  # per-chunk CRC-32 (METADATA extension line "crc32 ...")

    @property
    def n(self) -> int:
        return self.k + self.p

    @property
    def e(self) -> np.ndarray:
        return self.g[self.k :]


def write_metadata(path: str, total_size: int, p: int, k: int, e: np.ndarray | None, with_matrix: bool = True,
                   crc=None) -> None:
    lines = [f"{total_size}\n", f"{p} {k}\n"]
    if with_matrix:
        for i in range(k):
            lines.append("".join("1 " if i == j else "0 " for j in range(k)) + "\n")
        for i in range(p):
            lines.append("".join(f"{int(v)} " for v in np.asarray(e)[i]) + "\n")
        if crc:
            lines.append("crc32" + "".join(f" {int(c):08x}" for c in crc) + "\n")
    with open(path, "w") as f:
        f.writelines(lines)


def read_metadata(path: str) -> Metadata:
    with open(path) as f:
        toks = f.read().split()
    if len(toks) < 3:
        raise ValueError(f"malformed metadata {path}")
    total, p, k = int(toks[0]), int(toks[1]), int(toks[2])
    if k <= 0 or p < 0 or k + p > 256 or total < 0:
        raise ValueError(f"metadata out of range in {path}")
    vals = toks[3:]
    need = (k + p) * k
    if len(vals) == 0:
        g = GF256.generator(GF256.vandermonde_ref(k, p))
        return Metadata(total, p, k, g, False)
    if len(vals) < need:
        raise ValueError(f"truncated metadata matrix in {path}")
    g = np.array([int(v) for v in vals[:need]], dtype=np.int64)
    if g.min() < 0 or g.max() > 255:
        raise ValueError(f"metadata matrix entry out of range in {path}")
    crc = None
    rest = vals[need:]
    if rest and rest[0] == "crc32" and len(rest) >= 1 + k + p:
        crc = [int(h, 16) for h in rest[1 : 1 + k + p]]
    return Metadata(total, p, k, g.astype(np.uint8).reshape(k + p, k), True, crc)


def read_conf(path: str) -> list[str]:
    with open(path) as f:
        return f.read().split()


def write_conf(path: str, names) -> None:
    with open(path, "w") as f:
        f.writelines(f"{n}\n" for n in names)


def worst_case_conf(file: str, n: int, k: int) -> list[str]:
    """``src/unit-test.sh``: keep the last k chunks (erase natives 0..n-k-1)."""
    return [chunk_path(file, i) for i in range(n - k, n)]


def resolve_chunk(name: str, anchor: str) -> str:
    if os.path.exists(name) or os.path.isabs(name):
        return name
    alt = os.path.join(os.path.dirname(anchor), name)
    return alt if os.path.exists(alt) else name
