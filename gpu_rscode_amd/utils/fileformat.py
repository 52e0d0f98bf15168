"""The reference's on-disk formats, in Python.

* chunk files ``_<i>_<name>`` (``src/encode.cu:434-465``) — placed next to the input file, so
  paths with directories work (the reference breaks on them);
* ``<file>.METADATA``: ``totalSize\\n p k\\n`` then the k+p rows of ``G = [I; E]`` as ``"%d "``
  values (``src/encode.cu:61-101``); the CPU reference's 2-line form (``src/cpu-rs.c:465-476``) is
  accepted and G regenerated from the reference Vandermonde;
* decode config: whitespace-separated chunk names, row index ``atoi(basename + 1)``
  (``src/decode.cu:302-318``); ``worst_case_conf`` is ``src/unit-test.sh``;
* GF(2^16) stripes (extension; the reference's w = 16 field was never built): METADATA starts with
  a version line ``GFRS-METADATA 2 16`` and carries 16-bit matrix values; chunk sizes are rounded up
  to an even byte count (``csrc/include/gfrs/format.h``).

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


METADATA_VERSION = 2  # the versioned (GF(2^16)) form; unversioned = the reference's


def chunk_size(total: int, k: int, w: int = 8) -> int:
    c = max(1, (total + k - 1) // k)
    return (c + 1) // 2 * 2 if w == 16 else c


@dataclass
class Metadata:
    total_size: int
    p: int
    k: int
    g: np.ndarray  # (k+p) x k
    has_matrix: bool
    crc: list | None = None  # per-chunk CRC-32 (METADATA extension line "crc32 ...")
    w: int = 8  # field width: 8 (reference format) or 16 (versioned format, uint16 g)

    @property
    def n(self) -> int:
        return self.k + self.p

    @property
    def e(self) -> np.ndarray:
        return self.g[self.k :]


def write_metadata(path: str, total_size: int, p: int, k: int, e: np.ndarray | None, with_matrix: bool = True,
                   crc=None, w: int = 8) -> None:
    if w == 16 and not with_matrix:
        raise ValueError("the GF(2^16) METADATA always carries the matrix")
    lines = ([f"GFRS-METADATA {METADATA_VERSION} 16\n"] if w == 16 else []) + [f"{total_size}\n", f"{p} {k}\n"]
    if with_matrix:
        for i in range(k):
            lines.append("".join("1 " if i == j else "0 " for j in range(k)) + "\n")
        for i in range(p):
            lines.append("".join(f"{int(v)} " for v in np.asarray(e)[i]) + "\n")
        if crc:
            lines.append("crc32" + "".join(f" {int(c):08x}" for c in crc) + "\n")
    commit_file(path, "".join(lines).encode())


def _fsync_dir(path: str) -> None:
    try:
        fd = os.open(os.path.dirname(os.path.abspath(path)), os.O_RDONLY | os.O_DIRECTORY)
    except OSError:
        return
    try:
        os.fsync(fd)
    finally:
        os.close(fd)


def commit_file(path: str, data: bytes, durable: bool = True) -> None:
    """Durable, atomic replacement of a small file (the C++ ``gfrs::commit_file``): ``path.gfrs-tmp``
    written and fsync'ed, renamed over ``path``, the directory fsync'ed. A failed write (ENOSPC,
    EFBIG) raises and leaves ``path`` as it was — a METADATA exists only once complete."""
    tmp = path + ".gfrs-tmp"
    fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    try:
        view = memoryview(data)
        while view:
            view = view[os.write(fd, view):]
        if durable:
            os.fsync(fd)
    except BaseException:
        os.close(fd)
        os.unlink(tmp)
        raise
    os.close(fd)
    os.replace(tmp, path)
    if durable:
        _fsync_dir(path)


def remove_file(path: str, durable: bool = True) -> None:
    """Unlink ``path`` (missing is fine) and, durable, fsync its directory."""
    try:
        os.unlink(path)
    except FileNotFoundError:
        return
    if durable:
        _fsync_dir(path)


def read_metadata(path: str) -> Metadata:
    with open(path) as f:
        toks = f.read().split()
    w = 8
    if toks and toks[0] == "GFRS-METADATA":
        if len(toks) < 3 or toks[1] != str(METADATA_VERSION) or toks[2] != "16":
            raise ValueError(f"unsupported metadata version/field in {path}")
        w, toks = 16, toks[3:]
    if len(toks) < 3:
        raise ValueError(f"malformed metadata {path}")
    total, p, k = int(toks[0]), int(toks[1]), int(toks[2])
    if k <= 0 or p < 0 or k + p > (65535 if w == 16 else 256) or total < 0:
        raise ValueError(f"metadata out of range in {path}")
    vals = toks[3:]
    need = (k + p) * k
    if len(vals) == 0 and w == 8:
        g = GF256.generator(GF256.vandermonde_ref(k, p))
        return Metadata(total, p, k, g, False)
    if len(vals) < need:
        raise ValueError(f"truncated metadata matrix in {path}")
    g = np.array([int(v) for v in vals[:need]], dtype=np.int64)
    if g.min() < 0 or g.max() > (1 << w) - 1:
        raise ValueError(f"metadata matrix entry out of range in {path}")
    crc = None
    rest = vals[need:]
    if rest and rest[0] == "crc32" and len(rest) >= 1 + k + p:
        crc = [int(h, 16) for h in rest[1 : 1 + k + p]]
    dt = np.uint16 if w == 16 else np.uint8
    return Metadata(total, p, k, g.astype(dt).reshape(k + p, k), True, crc, w)


def read_conf(path: str) -> list[str]:
    with open(path) as f:
        return f.read().split()


def write_conf(path: str, names) -> None:
    commit_file(path, "".join(f"{n}\n" for n in names).encode(), durable=False)


def worst_case_conf(file: str, n: int, k: int) -> list[str]:
    """``src/unit-test.sh``: keep the last k chunks (erase natives 0..n-k-1)."""
    return [chunk_path(file, i) for i in range(n - k, n)]


def resolve_chunk(name: str, anchor: str) -> str:
    if os.path.exists(name) or os.path.isabs(name):
        return name
    alt = os.path.join(os.path.dirname(anchor), name)
    return alt if os.path.exists(alt) else name
