"""Multi-process stripe sharding over torch.distributed (gloo on CPU, world sizes 2 and 3).

The same code path runs over RCCL on MI355X (bench.py, N > 1); here it is exercised with the gloo
backend so the distributed logic is covered without a GPU.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gpu_rscode_amd.gf import GF256
from gpu_rscode_amd.parallel import dist as pdist


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fn_name):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    ctx = pdist.init_distributed(backend="gloo")
    try:
        globals()[fn_name](ctx)
    finally:
        dist.destroy_process_group()


def _run(fn_name, world=2):
    mp.spawn(_worker, args=(world, _free_port(), fn_name), nprocs=world, join=True)


def test_shard_range_partitions_and_aligns():
    for ncols in (1, 4095, 4096 * 7 + 3, 107374183):
        for world in (1, 2, 3, 8):
            spans = [pdist.shard_range(ncols, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == ncols
            for (a, b), (c, _) in zip(spans, spans[1:]):
                assert b == c and a % 4096 == 0


def _case_broadcast(ctx):
    e = GF256.vandermonde_ref(10, 4) if ctx.rank == 0 else None
    got = pdist.broadcast_matrix(e, ctx.device)
    assert np.array_equal(got, GF256.vandermonde_ref(10, 4))


def _case_scatter_gather(ctx):
    C = 3 * 4096 + 123
    full = torch.arange(5 * C, dtype=torch.int64).remainder(251).to(torch.uint8).view(5, C)
    shard = pdist.scatter_columns(full if ctx.rank == 0 else None, 5, C, ctx.device)
    a, b = pdist.shard_range(C, ctx.world, ctx.rank)
    assert torch.equal(shard, full[:, a:b])
    back = pdist.gather_columns(shard, C)
    if ctx.rank == 0:
        assert torch.equal(back, full)
    else:
        assert back is None


def _case_distributed_codec(ctx):
    k, n, C = 10, 14, 5 * 4096 + 77
    drs = pdist.DistributedRS(k, n, ctx)
    data = torch.from_numpy(np.random.default_rng(0).integers(0, 256, size=(k, C), dtype=np.uint8))
    parity = drs.encode_global(data if ctx.rank == 0 else None, C)
    if ctx.rank == 0:
        assert np.array_equal(parity.numpy(), GF256.gemm(GF256.vandermonde_ref(k, n - k), data.numpy()))
        stripe = torch.cat([data, parity])
        rows = [0, 1, 3, 5, 6, 8, 10, 11, 12, 13]
        surv = stripe[rows]
    else:
        rows, surv = None, None
    out = drs.decode_global(surv, rows, C)
    if ctx.rank == 0:
        assert torch.equal(out, data)


def _case_parity_exchange(ctx):
    """ParityExchange delivers exactly the senders' bytes: owners = piece `rank` of every rank's
    block, in source order; root = every peer's whole block on rank 0. Two alternating slots."""
    from gpu_rscode_amd.parallel.placement import ParityExchange, even_splits

    nbytes = 3 * 4096 + 17  # not divisible by the world size: uneven pieces

    def block(r, slot):
        return torch.arange(nbytes, dtype=torch.int64).add(7 * r + 131 * slot).remainder(251).to(torch.uint8)

    srcs = [block(ctx.rank, s) for s in range(2)]
    for mode in ("owners", "root", "none"):
        x = ParityExchange(srcs, mode)
        for slot in (0, 1, 0):
            x.start(slot)
            x.wait(slot)
            if mode == "owners":
                sp = even_splits(nbytes, ctx.world)
                off = sum(sp[: ctx.rank])
                mine = sp[ctx.rank]
                want = torch.cat([block(r, slot)[off:off + mine] for r in range(ctx.world)])
                assert torch.equal(x.recv, want), (mode, slot)
                assert x.bytes_sent == nbytes - mine and x.bytes_received == mine * (ctx.world - 1)
            elif mode == "root" and ctx.rank == 0:
                for r in range(1, ctx.world):
                    assert torch.equal(x.recv_list[r], block(r, slot)), (mode, slot, r)
            assert x.verify(slot)
        x.drain()


@pytest.mark.parametrize("case", ["_case_broadcast", "_case_scatter_gather", "_case_distributed_codec",
                                  "_case_parity_exchange"])
def test_distributed_world2(case):
    _run(case, 2)


def test_distributed_codec_world3():
    _run("_case_distributed_codec", 3)


def test_parity_exchange_world3():
    _run("_case_parity_exchange", 3)
