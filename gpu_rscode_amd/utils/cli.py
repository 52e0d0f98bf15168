"""Python CLI mirroring the reference's ``RS`` (``src/main.c:32-167``), plus a torch.distributed mode.

    python -m gpu_rscode_amd.utils.cli -k 4 -n 6 -e FILE [-s S] [-p G] [--backend gpu|cpu]
    python -m gpu_rscode_amd.utils.cli -d -i FILE -c CONF [-o OUT]
    torchrun --nproc-per-node 8 -m gpu_rscode_amd.utils.cli --dist -k 16 -n 20 -e FILE

Single-process modes call the native file codec (``csrc/io/codec_file.cpp``) with either the gfx950
streaming pipeline or the C++ CPU codec. ``--dist`` is the multi-GPU mode: every rank reads its own
4 KiB-aligned column range of every chunk straight from the file (no scatter) in bounded column
windows (``--window``, default 64 MiB per chunk row), encodes/decodes it on its GPU, and the results
are either gathered into rank 0 over RCCL point-to-point (default) or written in place by each rank
(``--gather none``, parallel pwrite).
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np


def _parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="gpu_rscode_amd", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-k", "-K", type=int, dest="k")
    ap.add_argument("-n", "-N", type=int, dest="n")
    ap.add_argument("-e", "-E", dest="encode_file")
    ap.add_argument("-d", "-D", action="store_true", dest="decode")
    ap.add_argument("-i", "-I", dest="in_file")
    ap.add_argument("-c", "-C", dest="conf")
    ap.add_argument("-o", "-O", dest="out", default="")
    ap.add_argument("-p", "-P", type=int, dest="grid", default=0, help="cap on gridDim.x (0 = uncapped)")
    ap.add_argument("-s", "-S", type=int, dest="streams", default=2, help="HIP streams per GPU")
    ap.add_argument("--backend", choices=["gpu", "cpu"], default=None)
    ap.add_argument("--matrix", default="vandermonde", choices=["vandermonde", "cauchy", "sys_vandermonde"])
    ap.add_argument("--cpu-meta", action="store_true", help="write the 2-line CPU-format METADATA")
    ap.add_argument("-w", "-W", "--field-width", type=int, choices=[8, 16], default=8, dest="field_w",
                    help="encode: symbol width, GF(2^8) or GF(2^16) (n <= 65535; decode reads it from METADATA)")
    ap.add_argument("--gpus", type=int, default=0, help="GPUs for the single-process pipeline (0 = all)")
    ap.add_argument("--slice", type=int, default=16 << 20)
    ap.add_argument("--zero-copy", action="store_true",
                    help="GPU backend: the GEMM kernel streams the pinned host rows over PCIe (no staging)")
    ap.add_argument("--threads", type=int, default=1, help="CPU backend threads")
    ap.add_argument("--mul", default="simd", help="CPU multiply strategy (row: the scalar product-row form)")
    ap.add_argument("--dist", action="store_true", help="torch.distributed multi-GPU mode (torchrun)")
    ap.add_argument("--gather", choices=["rccl", "none"], default="rccl")
    ap.add_argument("--window", type=int, default=None,
                    help="bounded-memory streaming codec: column windows of this many bytes per chunk "
                         "(0 = auto), checkpointed to <target>.PROGRESS and resumable")
    ap.add_argument("--no-resume", action="store_true", help="with --window: ignore a matching checkpoint")
    ap.add_argument("--no-sync", action="store_true", help="with --window: no fdatasync before checkpoints")
    ap.add_argument("-q", action="store_true", dest="quiet")
    return ap


def _say(a, msg):
    if not a.quiet:
        print(msg, flush=True)


def main(argv=None) -> int:
    a = _parser().parse_args(argv)
    if a.encode_file is None and not a.decode:
        _parser().print_help()
        return 2
    if a.dist:
        if a.field_w != 8:
            print("--dist runs GF(2^8) stripes; encode GF(2^16) in single-process mode", file=sys.stderr)
            return 2
        return _main_dist(a)
    from .._native import cpu, gpu_available, hip

    backend = a.backend or ("gpu" if gpu_available() else "cpu")
    if a.encode_file:
        if not a.k or not a.n or a.n < a.k:
            print("encode needs -k K -n N -e FILE with 1 <= K <= N", file=sys.stderr)
            return 2
        if a.field_w == 16 and (a.window is not None or a.cpu_meta):
            print("-w 16 writes the versioned METADATA without --window / --cpu-meta", file=sys.stderr)
            return 2
        fw = {} if a.field_w == 8 else dict(field_w=a.field_w)
        if a.zero_copy and backend == "gpu" and a.window is None:
            fw["zero_copy"] = True
        t = time.perf_counter()
        st = {} if a.window is None else dict(window=a.window, resume=not a.no_resume, durable=not a.no_sync)
        if backend == "gpu":
            ndev = hip().device_count()
            devs = list(range(a.gpus or ndev))
            fn = hip().encode_file_stream if st else hip().encode_file
            r = fn(a.encode_file, a.k, a.n - a.k, a.matrix, a.cpu_meta, devs, a.streams, a.slice, a.grid, **st, **fw)
        else:
            fn = cpu().encode_file_stream if st else cpu().encode_file
            r = fn(a.encode_file, a.k, a.n - a.k, a.matrix, a.cpu_meta, a.mul, a.threads, **st, **fw)
        if st:
            _say(a, f"Streamed {r['windows']} window(s) of {r['window']} bytes per chunk "
                    f"(resumed at {r['resumed_from']})")
        _say(a, f"Total {backend.upper()} encoding time: {r['ms_compute']:.3f}ms "
                f"({r['total_size'] / 1048576 / max(r['ms_compute'], 1e-9) * 1e3:.1f} MB/s; "
                f"wall {1e3 * (time.perf_counter() - t):.1f}ms incl. file I/O)")
        return 0
    if not a.in_file or not a.conf:
        print("decode needs -d -i FILE -c CONF", file=sys.stderr)
        return 2
    st = {} if a.window is None else dict(window=a.window, resume=not a.no_resume, durable=not a.no_sync)
    if backend == "gpu":
        ndev = hip().device_count()
        fn = hip().decode_file_stream if st else hip().decode_file
        zc = {"zero_copy": True} if (a.zero_copy and not st) else {}
        r = fn(a.in_file, a.conf, a.out, list(range(a.gpus or ndev)), a.streams, a.slice, a.grid, **st, **zc)
    else:
        fn = cpu().decode_file_stream if st else cpu().decode_file
        r = fn(a.in_file, a.conf, a.out, a.mul, a.threads, **st)
    _say(a, f"Total {backend.upper()} decoding time: {r['ms_compute']:.3f}ms ({r['erased']} erased native chunk(s))")
    return 0


# ---- distributed mode -------------------------------------------------------------------------
DIST_WINDOW = 64 << 20  # default column window per chunk row and rank (host RAM ~ (k + p) x window)


def _read_cols(path: str, offset: int, nbytes: int, out: np.ndarray) -> None:
    """pread ``nbytes`` at ``offset`` into ``out``; zero-fill the rest (past EOF / past nbytes)."""
    got = 0
    if nbytes > 0:
        fd = os.open(path, os.O_RDONLY)
        try:
            view = memoryview(out)[:nbytes]
            while got < nbytes:
                n = os.preadv(fd, [view[got:]], offset + got)
                if n <= 0:
                    break
                got += n
        finally:
            os.close(fd)
    out[got:] = 0


def _pwrite(fd: int, offset: int, data: np.ndarray) -> None:
    view = memoryview(np.ascontiguousarray(data)).cast("B")
    done = 0
    while done < len(view):
        done += os.pwrite(fd, view[done:], offset + done)


def _windows(world: int, C: int, window: int):
    """Per window index t: every rank's (column offset, width) — identical on all ranks, so the
    collective per window lines up even where a rank's shard is exhausted (width 0)."""
    from ..parallel.dist import shard_range

    spans = [shard_range(C, world, r) for r in range(world)]
    nwin = max(((b - a) + window - 1) // window for a, b in spans) if C else 0
    for t in range(nwin):
        yield [(a + t * window, max(0, min(window, b - a - t * window))) for a, b in spans]


def _main_dist(a) -> int:
    """Windowed, column-sharded encode/decode over torch.distributed.

    Every rank owns a 4 KiB-aligned column range of every chunk (the reference's per-device split,
    src/encode.cu:368-381) and walks it in windows of ``--window`` bytes per chunk row, so host
    memory stays bounded at ~(k + p) x window per rank whatever the file size. Per window: pread
    of the rank's columns, H2D, GF-GEMM on the rank's GPU, then either every rank pwrites its own
    columns (``--gather none``) or the window's results travel to rank 0 over RCCL point-to-point
    (received in place, one xGMI link per peer) and rank 0 writes them (``--gather rccl``, the
    reference's gather-to-one-writer, src/encode.cu:410-429). Rank 0 creates every output at its
    final size first, so no stale bytes of an older, longer file survive."""
    import torch
    import torch.distributed as dist

    from ..models import ReedSolomon
    from ..parallel.dist import broadcast_matrix, gather_pieces, init_distributed
    from . import fileformat as ff

    ctx = init_distributed()
    world, rank = ctx.world, ctx.rank
    window = max(4096, ((a.window or DIST_WINDOW) + 4095) // 4096 * 4096)
    t0 = time.perf_counter()

    def barrier():
        if world > 1:
            dist.barrier()

    def create(path: str, size: int) -> None:
        fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        try:
            os.ftruncate(fd, size)
        finally:
            os.close(fd)

    if a.encode_file:
        path = a.encode_file
        total = os.path.getsize(path)
        k, p = a.k, a.n - a.k
        C = ff.chunk_size(total, k)
        e = ReedSolomon(k, a.n, matrix=a.matrix).E if ctx.is_root else None
        e = broadcast_matrix(e, ctx.device)
        rs = ReedSolomon(k, a.n)
        rs.E, rs.G = e, np.vstack([np.eye(k, dtype=np.uint8), e])
        if ctx.is_root:
            for i in range(a.n):
                create(ff.chunk_path(path, i), C)
        barrier()
        fds = [os.open(ff.chunk_path(path, i), os.O_WRONLY) for i in range(a.n)]
        host = np.zeros((k, window), dtype=np.uint8)
        try:
            for spans in _windows(world, C, window):
                o, w = spans[rank]
                if w:
                    for j in range(k):  # natives: this rank's columns of chunk j, zero past EOF
                        start = j * C + o
                        _read_cols(path, start, max(0, min(w, total - start)), host[j, :w])
                        _pwrite(fds[j], o, host[j, :w])
                    parity = rs.encode(torch.from_numpy(host[:, :w]).to(ctx.device))
                else:
                    parity = torch.empty((p, 0), dtype=torch.uint8, device=ctx.device)
                if a.gather == "rccl" and world > 1:
                    if ctx.device.type == "cuda":
                        torch.cuda.synchronize()
                    full = gather_pieces(parity, [ww for _, ww in spans])
                    if ctx.is_root:
                        ph = full.cpu().numpy()
                        col = 0
                        for ro, rw in spans:
                            for i in range(p):
                                _pwrite(fds[k + i], ro, ph[i, col:col + rw])
                            col += rw
                elif w:
                    ph = parity.cpu().numpy()
                    for i in range(p):
                        _pwrite(fds[k + i], o, ph[i, :w])
        finally:
            for fd in fds:
                os.close(fd)
        if ctx.is_root:
            ff.write_metadata(ff.metadata_path(path), total, p, k, e, with_matrix=not a.cpu_meta)
        barrier()
        lo, hi = spans_of(world, C, rank)
        _say(a, f"[rank {rank}] encoded columns [{lo}, {hi}) in windows of {window} B "
                f"in {1e3 * (time.perf_counter() - t0):.1f}ms")
    else:
        md = ff.read_metadata(ff.metadata_path(a.in_file))
        if md.w != 8:
            raise SystemExit("--dist decodes GF(2^8) stripes; decode a GF(2^16) stripe in single-process mode")
        names = ff.read_conf(a.conf)[: md.k]
        rows = [ff.chunk_index(nm) for nm in names]
        k, C = md.k, ff.chunk_size(md.total_size, md.k)
        rs = ReedSolomon(k, md.n)
        rs.E, rs.G = md.e, md.g
        dst = a.out or a.in_file
        if ctx.is_root:
            create(dst, md.total_size)
        barrier()
        paths = [ff.resolve_chunk(nm, a.in_file) for nm in names]
        fd_out = os.open(dst, os.O_WRONLY)
        host = np.zeros((k, window), dtype=np.uint8)

        def write_natives(nat: np.ndarray, o: int, w: int) -> None:
            for j in range(k):
                start = j * C + o
                n = max(0, min(w, md.total_size - start))
                if n:
                    _pwrite(fd_out, start, nat[j, :n])

        try:
            for spans in _windows(world, C, window):
                o, w = spans[rank]
                if w:
                    for j, pth in enumerate(paths):
                        _read_cols(pth, o, w, host[j, :w])
                    out = rs.decode(torch.from_numpy(host[:, :w]).to(ctx.device), rows)
                else:
                    out = torch.empty((k, 0), dtype=torch.uint8, device=ctx.device)
                if a.gather == "rccl" and world > 1:
                    if ctx.device.type == "cuda":
                        torch.cuda.synchronize()
                    full = gather_pieces(out, [ww for _, ww in spans])
                    if ctx.is_root:
                        fh = full.cpu().numpy()
                        col = 0
                        for ro, rw in spans:
                            write_natives(fh[:, col:col + rw], ro, rw)
                            col += rw
                elif w:
                    write_natives(out.cpu().numpy(), o, w)
        finally:
            os.close(fd_out)
        barrier()
        lo, hi = spans_of(world, C, rank)
        _say(a, f"[rank {rank}] decoded columns [{lo}, {hi}) in windows of {window} B "
                f"in {1e3 * (time.perf_counter() - t0):.1f}ms")
    if world > 1:
        dist.destroy_process_group()
    return 0


def spans_of(world: int, C: int, rank: int) -> tuple[int, int]:
    from ..parallel.dist import shard_range

    return shard_range(C, world, rank)


if __name__ == "__main__":
    sys.exit(main())
