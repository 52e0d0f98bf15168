"""Python CLI mirroring the reference's ``RS`` (``src/main.c:32-167``), plus a torch.distributed mode.

    python -m gpu_rscode_amd.utils.cli -k 4 -n 6 -e FILE [-s S] [-p G] [--backend gpu|cpu]
    python -m gpu_rscode_amd.utils.cli -d -i FILE -c CONF [-o OUT]
    torchrun --nproc-per-node 8 -m gpu_rscode_amd.utils.cli --dist -k 16 -n 20 -e FILE

Single-process modes call the native file codec (``csrc/io/codec_file.cpp``) with either the gfx950
streaming pipeline or the C++ CPU codec. ``--dist`` is the multi-GPU mode (one rank per GPU): every
rank streams its own 4 KiB-aligned column range of every chunk through the native windowed codec
(``csrc/io/stream_codec.cpp``, shard mode: read / GEMM / write overlapped, pinned buffers,
checkpointed per shard), reading its columns straight from the file and writing them straight into
the outputs; only the survivor choice and the per-chunk CRC-32s cross the process group.
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
    ap.add_argument("--pg-timeout", type=float, default=None,
                    help="--dist: process-group timeout in seconds (a lost peer ends the job after at most this; "
                         "default GFRS_PG_TIMEOUT_S or 300, parallel.dist.default_pg_timeout)")
    ap.add_argument("--window", type=int, default=None,
                    help="bounded-memory streaming codec: column windows of this many bytes per chunk "
                         "(0 = auto), checkpointed to <target>.PROGRESS and resumable")
    ap.add_argument("--no-resume", action="store_true", help="with --window: ignore a matching checkpoint")
    ap.add_argument("--no-sync", action="store_true", help="with --window: no fdatasync before checkpoints")
    ap.add_argument("-q", action="store_true", dest="quiet")
    ap.add_argument("--json", action="store_true", help="--dist: rank 0 prints a JSON line of the job's codec time")
    # testing: a shard stops after this many windows (a simulated crash; the job fails and a re-run resumes)
    ap.add_argument("--stop-after", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--stop-rank", type=int, default=-1, help=argparse.SUPPRESS)
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
        if a.field_w == 16 and a.cpu_meta:
            print("-w 16 writes the versioned METADATA (no --cpu-meta form)", file=sys.stderr)
            return 2
        fw = {} if a.field_w == 8 else dict(field_w=a.field_w)
        if a.zero_copy and backend == "gpu":
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
        zc = {"zero_copy": True} if a.zero_copy else {}
        r = fn(a.in_file, a.conf, a.out, list(range(a.gpus or ndev)), a.streams, a.slice, a.grid, **st, **zc)
    else:
        fn = cpu().decode_file_stream if st else cpu().decode_file
        r = fn(a.in_file, a.conf, a.out, a.mul, a.threads, **st)
    _say(a, f"Total {backend.upper()} decoding time: {r['ms_compute']:.3f}ms ({r['erased']} erased native chunk(s))")
    return 0


# ---- distributed mode -------------------------------------------------------------------------
def _size_file(path: str, size: int) -> bool:
    """Create ``path`` if missing and set its size to exactly ``size`` (shards then write their
    columns in place; an older, longer file loses its stale tail). Never truncated to zero first:
    the columns a resumed shard checkpointed before a crash are still in it, and every column no
    checkpoint covers is rewritten by its shard. Returns whether the file was already there at
    exactly that size — when one was not, no checkpoint may be trusted (a re-created file is zeros
    where a checkpoint says columns were written)."""
    try:
        intact = os.stat(path).st_size == size
    except FileNotFoundError:
        intact = False
    fd = os.open(path, os.O_WRONLY | os.O_CREAT, 0o644)
    try:
        os.ftruncate(fd, size)
    finally:
        os.close(fd)
    return intact


def _shard_checkpoints(target: str, C: int, world: int) -> list[str]:
    from .._native import cpu
    from ..parallel.dist import shard_range

    return [cpu().shard_progress_path(target, *shard_range(C, world, r)) for r in range(world)]


def _prune_checkpoints(target: str, keep: list[str]) -> None:
    """Rank 0, before any shard starts: remove every ``<target>.PROGRESS.*`` that is not one of this
    job's shard checkpoints (another world size or chunk size, an interrupted temp file), so no stale
    checkpoint can ever be matched later."""
    from .._native import cpu

    prefix = os.path.basename(cpu().progress_path(target)) + "."
    d = os.path.dirname(os.path.abspath(target))
    keep_names = {os.path.basename(x) for x in keep}
    for name in os.listdir(d):
        if name.startswith(prefix) and name not in keep_names:
            try:
                os.unlink(os.path.join(d, name))
            except FileNotFoundError:
                pass


def _interrupted(a, rank: int, r: dict) -> None:
    if not r["complete"]:
        raise RuntimeError(f"shard stopped after {r['windows']} window(s) (--stop-after {a.stop_after}); "
                           "its checkpoint resumes it")


def _stop_after(a, rank: int) -> int:
    return a.stop_after if a.stop_after >= 0 and a.stop_rank in (-1, rank) else -1


def _main_dist(a) -> int:
    """Multi-GPU file codec: one rank per GPU (torchrun), each running its column shard through the
    native streaming codec.

    The reference splits every chunk's columns over its GPUs (src/encode.cu:368-381,
    src/decode.cu:335-408), stages the slices through pinned host buffers and gathers the results
    into one writer (src/encode.cu:389-398, 410-429). Here every rank owns a 4 KiB-aligned column
    range of every chunk (``shard_range``) and streams it through ``encode_file_stream`` /
    ``decode_file_stream`` in shard mode — the three-stage read / GEMM / write window pipeline of
    ``csrc/io/stream_codec.cpp`` with pinned buffers on its own GPU, checkpointed per shard — reading
    its columns straight from the input file and pwriting them straight into the outputs. What
    crosses the process group is tiny: rank 0 creates the outputs at their final size, picks and
    combines every rank's per-chunk CRC-32s (``crc32_combine`` in column order) into the METADATA
    (encode), and checks the decode survivors the same way: each rank CRCs only its column shard of
    every candidate, rank 0 combines and picks, and the choice is broadcast.

    A rank that fails exits non-zero at once, issuing no further collective: its peers' next one
    fails (gloo) or is aborted by the process group's bounded timeout (``--pg-timeout``), and torchrun
    ends the job."""
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # (before the first HIP call: RCCL peers)
    from ..parallel.dist import default_pg_timeout, init_distributed

    ctx = init_distributed(timeout_s=default_pg_timeout() if a.pg_timeout is None else a.pg_timeout)
    try:
        rc = _dist_run(a, ctx)
    except Exception as ex:  # noqa: BLE001 — this rank stops here, without another collective
        print(f"[rank {ctx.rank}] --dist failed: {type(ex).__name__}: {ex}", file=sys.stderr, flush=True)
        sys.stdout.flush()
        os._exit(1)
    import torch.distributed as dist

    if dist.is_initialized():
        dist.destroy_process_group()
    return rc


def _dist_run(a, ctx) -> int:
    import torch
    import torch.distributed as dist

    from .._native import cpu, hip
    from ..models import ReedSolomon
    from ..parallel.dist import shard_range
    from . import fileformat as ff

    world, rank = ctx.world, ctx.rank
    on_gpu = ctx.device.type == "cuda"

    def barrier():
        if world > 1:
            dist.barrier()

    fault = os.environ.get("GFRS_DIST_FAULT_RANK")
    t0 = time.perf_counter()
    st = dict(window=a.window or 0, resume=not a.no_resume, durable=not a.no_sync)
    if a.encode_file:
        path = a.encode_file
        if not a.k or not a.n or a.n < a.k:
            raise ValueError("encode needs -k K -n N -e FILE with 1 <= K <= N")
        if a.field_w == 16 and a.cpu_meta:
            raise ValueError("-w 16 writes the versioned METADATA (no --cpu-meta form)")
        total = os.path.getsize(path)
        k, p, n = a.k, a.n - a.k, a.n
        C = max(2 if a.field_w == 16 else 1, ff.chunk_size(total, k, a.field_w))
        # the device setup (streams, buffers, code object) runs on a helper thread from here on,
        # under the output creation, the barrier and the first window's reads (as bin/RS overlaps it)
        prep = (hip().prepare_encode_async(path, k, p, [ctx.local_rank], a.streams, a.slice, a.grid, a.field_w,
                                           a.zero_copy, a.window or 0) if on_gpu else None)
        # Commit protocol (a crash anywhere leaves either no METADATA or a complete stripe, and a
        # re-run resumes): rank 0 removes an older METADATA, keeps this layout's shard checkpoints
        # (unless --no-resume) and sizes the chunks without truncating them; every shard resumes from
        # its own checkpoint; rank 0 commits the METADATA atomically; only then do the shards drop
        # their checkpoints.
        ckpts = _shard_checkpoints(path, C, world)
        if ctx.is_root:
            ff.remove_file(ff.metadata_path(path))
            intact = all([_size_file(ff.chunk_path(path, i), C) for i in range(n)])
            _prune_checkpoints(path, ckpts if intact and not a.no_resume else [])
        barrier()
        if fault is not None and int(fault) == rank:
            raise RuntimeError("injected fault (GFRS_DIST_FAULT_RANK)")
        lo, hi = shard_range(C, world, rank)
        kw = dict(st, field_w=a.field_w, col_lo=lo, col_hi=hi, shard=True, stop_after=_stop_after(a, rank))
        if on_gpu:
            r = hip().encode_file_stream(path, k, p, a.matrix, a.cpu_meta, [ctx.local_rank], a.streams, a.slice,
                                         a.grid, zero_copy=a.zero_copy, prep=prep, **kw)
        else:
            r = cpu().encode_file_stream(path, k, p, a.matrix, a.cpu_meta, a.mul, a.threads, **kw)
        _interrupted(a, rank, r)
        # every rank's shard CRCs (and width) to rank 0, combined in column order
        mine = torch.tensor([hi - lo] + list(r["crc"]), dtype=torch.int64, device=ctx.device)
        parts = [torch.zeros_like(mine) for _ in range(world)] if world > 1 else [mine]
        if world > 1:
            dist.all_gather(parts, mine)
        if ctx.is_root:
            crc = [0] * n
            for part in parts:
                vals = part.tolist()
                crc = [cpu().crc32_combine(c, int(x), vals[0]) for c, x in zip(crc, vals[1:])]
            e = ReedSolomon(k, n, matrix=a.matrix, field="gf65536" if a.field_w == 16 else "gf256").E
            ff.write_metadata(ff.metadata_path(path), total, p, k, e, with_matrix=not a.cpu_meta,
                              crc=None if a.cpu_meta else crc, w=a.field_w)
        barrier()
        ff.remove_file(ckpts[rank], durable=not a.no_sync)  # (the METADATA is committed)
        _say(a, f"[rank {rank}] encoded columns [{lo}, {hi}) of {C} in {r['windows']} window(s) of {r['window']} B "
                f"in {1e3 * (time.perf_counter() - t0):.1f}ms (read {r['ms_read']:.1f}, GEMM {r['ms_compute']:.1f}, "
                f"write {r['ms_write']:.1f} ms, overlapped)")
        _dist_summary(a, ctx, "encode", total, t0)
        return 0
    if not a.in_file or not a.conf:
        raise ValueError("decode needs -d -i FILE -c CONF")
    md = ff.read_metadata(ff.metadata_path(a.in_file))
    C = max(2 if md.w == 16 else 1, ff.chunk_size(md.total_size, md.k, md.w))
    dst = a.out or a.in_file
    # device setup under the survivor choice (the survivors' bytes are read and CRC-checked first)
    prep = (hip().prepare_decode_async(a.in_file, [ctx.local_rank], a.streams, a.slice, a.grid, a.zero_copy,
                                       a.window or 0) if on_gpu else None)
    lo, hi = shard_range(C, world, rank)
    # The survivor check, split over the ranks: each reads and CRCs only its column shard of the
    # conf candidates; rank 0 combines the CRCs in column order, compares them with the METADATA and
    # picks (one rank: the whole check in-process). Round 1 reads the first k candidates only (all
    # a clean decode needs, as the single-process check); a round 2 over the rest runs only when
    # rank 0 finds those short of a recoverable set. pick[0]: 0 = chosen, 1 = failed, 2 = read more.
    ckpts = _shard_checkpoints(dst, C, world)
    pick = torch.zeros(md.k + 1, dtype=torch.int64, device=ctx.device)
    err = None
    verdicts = None
    for first, count in ((0, md.k), (md.k, -1)):
        parts = None
        if world > 1:
            n = md.k + md.p
            rows_h = [[1, 0, 0]] + [[0, 0, 0]] * n  # row 0: status, candidate count, shard width
            try:
                got = cpu().shard_crcs(a.in_file, a.conf, lo, hi, first, count)
                rows_h[0] = [0, len(got), hi - lo]
                for i, (idx, present, crc) in enumerate(got[:n]):
                    rows_h[1 + i] = [idx, int(present), crc]
            except Exception:  # noqa: BLE001 — rank 0 reports (it hits the same conf / METADATA)
                rows_h[0][0] = 1
            shard = torch.tensor(rows_h, dtype=torch.int64).to(ctx.device)
            parts = [torch.zeros_like(shard) for _ in range(world)]
            dist.all_gather(parts, shard)
        if ctx.is_root:
            pick.zero_()
            try:
                if parts is None:
                    rows, _ = cpu().choose_survivors(a.in_file, a.conf)
                else:
                    got_v = _combine_shard_crcs(parts, md)
                    verdicts = got_v if verdicts is None else [x | y for x, y in zip(verdicts, got_v)]
                    rows = cpu().choose_survivors_given(a.in_file, a.conf, verdicts)
                pick[1:] = torch.tensor(rows, dtype=torch.int64)
            except Exception as ex:  # noqa: BLE001 — told to every rank through the broadcast
                more = parts is not None and first == 0 and verdicts is not None and len(verdicts) > md.k
                pick[0] = 2 if more else 1
                err = ex
            if not int(pick[0].item()):
                intact = _size_file(dst, md.total_size)
                _prune_checkpoints(dst, ckpts if intact and not a.no_resume else [])
        if world > 1:
            dist.broadcast(pick, 0)
        if int(pick[0].item()) != 2:
            break
    if int(pick[0].item()):
        if ctx.is_root:
            raise err
        raise RuntimeError("rank 0 could not choose the decode survivors")
    rows = [int(x) for x in pick[1:].tolist()]
    barrier()
    if fault is not None and int(fault) == rank:
        raise RuntimeError("injected fault (GFRS_DIST_FAULT_RANK)")
    kw = dict(st, col_lo=lo, col_hi=hi, shard=True, rows=rows, stop_after=_stop_after(a, rank))
    if on_gpu:
        r = hip().decode_file_stream(a.in_file, a.conf, dst, [ctx.local_rank], a.streams, a.slice, a.grid,
                                     zero_copy=a.zero_copy, prep=prep, **kw)
    else:
        r = cpu().decode_file_stream(a.in_file, a.conf, dst, a.mul, a.threads, **kw)
    _interrupted(a, rank, r)
    barrier()
    ff.remove_file(ckpts[rank], durable=not a.no_sync)  # (every shard of the output is written)
    _say(a, f"[rank {rank}] decoded columns [{lo}, {hi}) of {C} ({r['erased']} erased native(s)) in "
            f"{r['windows']} window(s) of {r['window']} B in {1e3 * (time.perf_counter() - t0):.1f}ms")
    _dist_summary(a, ctx, "decode", md.total_size, t0)
    return 0


def _combine_shard_crcs(parts, md) -> list:
    """Every conf candidate's verdict (1 = usable) from the ranks' shard reports (``shard_crcs``:
    row 0 = status, candidate count, shard width; then chunk index, present, CRC-32 of the shard):
    present on every rank, and the shard CRCs combined in rank (= column) order equal to the
    METADATA's (METADATA without CRCs: present is enough)."""
    from .._native import cpu

    heads = [p[0].tolist() for p in parts]
    if any(h[0] for h in heads):
        raise RuntimeError("a rank could not read the survivors' configuration or METADATA")
    ncand = int(heads[0][1])
    rows = [p[1:1 + ncand].tolist() for p in parts]
    intact = []
    for ci in range(ncand):
        idx = int(rows[0][ci][0])
        present = all(int(r[ci][1]) for r in rows)
        crc = 0
        for r, h in zip(rows, heads):
            crc = cpu().crc32_combine(crc, int(r[ci][2]), int(h[2]))
        ok = present and (not md.crc or crc == md.crc[idx])
        intact.append(1 if ok else 0)
    return intact


def _dist_summary(a, ctx, op: str, size: int, t0: float) -> None:
    """``--json``: rank 0 prints one line with the job's codec time: max over ranks from the moment
    the process group exists (outputs created, survivors chosen and CRC-verified, every shard
    streamed, CRCs combined, METADATA written) to the final barrier — the part bin/RS reports as its
    file codec time."""
    if not a.json:
        return
    import json

    import torch
    import torch.distributed as dist

    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=ctx.device)
    if ctx.world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if ctx.is_root:
        codec_s = float(t.item())
        print(json.dumps({"op": op, "ranks": ctx.world, "bytes": size, "codec_ms": round(codec_s * 1e3, 3),
                          "codec_GBps": round(size / codec_s / 1e9, 3)}), flush=True)


def spans_of(world: int, C: int, rank: int) -> tuple[int, int]:
    from ..parallel.dist import shard_range

    return shard_range(C, world, rank)


if __name__ == "__main__":
    sys.exit(main())
