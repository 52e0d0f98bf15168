"""Python CLI mirroring the reference's ``RS`` (``src/main.c:32-167``), plus a torch.distributed mode.

    python -m gpu_rscode_amd.utils.cli -k 4 -n 6 -e FILE [-s S] [-p G] [--backend gpu|cpu]
    python -m gpu_rscode_amd.utils.cli -d -i FILE -c CONF [-o OUT]
    torchrun --nproc-per-node 8 -m gpu_rscode_amd.utils.cli --dist -k 16 -n 20 -e FILE

Single-process modes call the native file codec (``csrc/io/codec_file.cpp``) with either the gfx950
streaming pipeline or the C++ CPU codec. ``--dist`` is the multi-GPU mode: every rank reads its own
4 KiB-aligned column range of every chunk straight from the file (no scatter), encodes/decodes it
on its GPU, and the results are either gathered into rank 0 over RCCL point-to-point (default) or
written in place by each rank (``--gather none``, parallel pwrite).
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
    ap.add_argument("--gpus", type=int, default=0, help="GPUs for the single-process pipeline (0 = all)")
    ap.add_argument("--slice", type=int, default=16 << 20)
    ap.add_argument("--threads", type=int, default=1, help="CPU backend threads")
    ap.add_argument("--mul", default="row", help="CPU multiply strategy")
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
        return _main_dist(a)
    from .._native import cpu, gpu_available, hip

    backend = a.backend or ("gpu" if gpu_available() else "cpu")
    if a.encode_file:
        if not a.k or not a.n or a.n < a.k:
            print("encode needs -k K -n N -e FILE with 1 <= K <= N", file=sys.stderr)
            return 2
        t = time.perf_counter()
        st = {} if a.window is None else dict(window=a.window, resume=not a.no_resume, durable=not a.no_sync)
        if backend == "gpu":
            ndev = hip().device_count()
            devs = list(range(a.gpus or ndev))
            fn = hip().encode_file_stream if st else hip().encode_file
            r = fn(a.encode_file, a.k, a.n - a.k, a.matrix, a.cpu_meta, devs, a.streams, a.slice, a.grid, **st)
        else:
            fn = cpu().encode_file_stream if st else cpu().encode_file
            r = fn(a.encode_file, a.k, a.n - a.k, a.matrix, a.cpu_meta, a.mul, a.threads, **st)
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
        r = fn(a.in_file, a.conf, a.out, list(range(a.gpus or ndev)), a.streams, a.slice, a.grid, **st)
    else:
        fn = cpu().decode_file_stream if st else cpu().decode_file
        r = fn(a.in_file, a.conf, a.out, a.mul, a.threads, **st)
    _say(a, f"Total {backend.upper()} decoding time: {r['ms_compute']:.3f}ms ({r['erased']} erased native chunk(s))")
    return 0


# ---- distributed mode -------------------------------------------------------------------------
def _read_cols(path: str, offset: int, nbytes: int, out: np.ndarray) -> None:
    """pread ``nbytes`` at ``offset`` into ``out``; zero-fill past EOF."""
    out[:] = 0
    if nbytes <= 0:
        return
    with open(path, "rb") as f:
        f.seek(offset)
        buf = f.read(nbytes)
    out[: len(buf)] = np.frombuffer(buf, dtype=np.uint8)


def _pwrite(path: str, offset: int, data: np.ndarray) -> None:
    fd = os.open(path, os.O_WRONLY | os.O_CREAT, 0o644)
    try:
        os.pwrite(fd, data.tobytes(), offset)
    finally:
        os.close(fd)


def _main_dist(a) -> int:
    import torch
    import torch.distributed as dist

    from ..models import ReedSolomon
    from ..parallel.dist import broadcast_matrix, gather_columns, init_distributed, shard_range
    from . import fileformat as ff

    ctx = init_distributed()
    world, rank = ctx.world, ctx.rank
    t0 = time.perf_counter()
    if a.encode_file:
        path = a.encode_file
        total = os.path.getsize(path)
        k, p = a.k, a.n - a.k
        C = ff.chunk_size(total, k)
        e = ReedSolomon(k, a.n, matrix=a.matrix).E if ctx.is_root else None
        e = broadcast_matrix(e, ctx.device)
        lo, hi = shard_range(C, world, rank)
        host = np.zeros((k, hi - lo), dtype=np.uint8)
        for j in range(k):  # each rank reads its own columns of every native chunk: no scatter
            start = j * C + lo
            _read_cols(path, start, max(0, min(hi - lo, total - start)), host[j])
        rs = ReedSolomon(k, a.n)
        rs.E, rs.G = e, np.vstack([np.eye(k, dtype=np.uint8), e])
        data = torch.from_numpy(host).to(ctx.device)
        parity = rs.encode(data)
        if ctx.device.type == "cuda":
            torch.cuda.synchronize()
        if a.gather == "rccl":
            full = gather_columns(parity.contiguous(), C)
            if ctx.is_root:
                fullh = full.cpu().numpy()
                with open(path, "rb") as f:
                    blob = f.read()
                for j in range(k):
                    seg = np.zeros(C, dtype=np.uint8)
                    chunk = np.frombuffer(blob[j * C : (j + 1) * C], dtype=np.uint8)
                    seg[: len(chunk)] = chunk
                    seg.tofile(ff.chunk_path(path, j))
                for i in range(p):
                    fullh[i].tofile(ff.chunk_path(path, k + i))
        else:
            ph = parity.cpu().numpy()
            for j in range(k):
                _pwrite(ff.chunk_path(path, j), lo, host[j])
            for i in range(p):
                _pwrite(ff.chunk_path(path, k + i), lo, ph[i])
        if ctx.is_root:
            ff.write_metadata(ff.metadata_path(path), total, p, k, e, with_matrix=not a.cpu_meta)
        if world > 1:
            dist.barrier()
        _say(a, f"[rank {rank}] encoded columns [{lo}, {hi}) in {1e3 * (time.perf_counter() - t0):.1f}ms")
    else:
        md = ff.read_metadata(ff.metadata_path(a.in_file))
        names = ff.read_conf(a.conf)[: md.k]
        rows = [ff.chunk_index(nm) for nm in names]
        k, C = md.k, ff.chunk_size(md.total_size, md.k)
        lo, hi = shard_range(C, world, rank)
        host = np.zeros((k, hi - lo), dtype=np.uint8)
        for j, nm in enumerate(names):
            _read_cols(ff.resolve_chunk(nm, a.in_file), lo, hi - lo, host[j])
        rs = ReedSolomon(k, md.n)
        rs.E, rs.G = md.e, md.g
        out = rs.decode(torch.from_numpy(host).to(ctx.device), rows)
        if ctx.device.type == "cuda":
            torch.cuda.synchronize()
        dst = a.out or a.in_file
        if a.gather == "rccl":
            full = gather_columns(out.contiguous(), C)
            if ctx.is_root:
                full.cpu().numpy().reshape(-1)[: md.total_size].tofile(dst)
        else:
            oh = out.cpu().numpy()
            if ctx.is_root:
                with open(dst, "wb") as f:
                    f.truncate(md.total_size)
            if world > 1:
                dist.barrier()
            for j in range(k):
                start = j * C + lo
                n = max(0, min(hi - lo, md.total_size - start))
                if n:
                    _pwrite(dst, start, oh[j, :n])
        if world > 1:
            dist.barrier()
        _say(a, f"[rank {rank}] decoded columns [{lo}, {hi}) in {1e3 * (time.perf_counter() - t0):.1f}ms")
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
