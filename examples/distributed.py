#!/usr/bin/env python3
"""Multi-rank tour: the reference's multi-GPU encode/decode (one stripe column-sharded over the
devices, src/encode.cu:357-432, src/decode.cu:335-408) as torch.distributed ranks, and a decode
whose erasure pattern is broadcast by rank 0 straight into every rank's device memory.

  torchrun --nproc-per-node N --master-addr 127.0.0.1 examples/distributed.py   (one rank per GPU)
  python examples/distributed.py    (no torchrun: a one-rank RCCL group on a GPU, or 2 gloo ranks on the CPU)
"""
from __future__ import annotations

import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from gpu_rscode_amd.gf import GF256  # noqa: E402
from gpu_rscode_amd.parallel import DistributedRS, init_distributed  # noqa: E402


def tour(force_pg: bool) -> None:
    ctx = init_distributed(force_pg=force_pg)
    k, n, C = 10, 14, 3 * 4096 + 1001  # odd C, as the reference's 1 GiB / k = 10 stripe
    drs = DistributedRS(k, n, ctx)  # E comes from rank 0 (broadcast)
    host = np.random.default_rng(7).integers(0, 256, size=(k, C), dtype=np.uint8)
    data = torch.from_numpy(host).to(ctx.device) if ctx.is_root else None

    # encode: rank 0's stripe -> column shards (point-to-point) -> parity gathered in place on rank 0
    parity = drs.encode_global(data, C)
    rows = [0, 1, 3, 5, 6, 8, 10, 11, 12, 13]  # natives 2, 4, 7, 9 lost
    if ctx.is_root:
        assert np.array_equal(parity.cpu().numpy(), GF256.gemm(drs.rs.E, host)), "parity mismatch"
        surv = torch.cat([data, parity.contiguous()])[rows].contiguous()
    else:
        surv = None
    out = drs.decode_global(surv, rows if ctx.is_root else None, C)
    if ctx.is_root:
        assert np.array_equal(out.cpu().numpy(), host), "decode mismatch"

    if ctx.device.type == "cuda":
        # every rank encodes its own stripe; rank 0 decides which chunks are lost and broadcasts the
        # survivor list into each rank's device-built decode plan (no host round trip on the others)
        from gpu_rscode_amd import ReedSolomon, alloc_rows
        from gpu_rscode_amd.ops import PatternDecoder

        rs = ReedSolomon(k, n)
        mine = np.random.default_rng(100 + ctx.rank).integers(0, 256, size=(k, C), dtype=np.uint8)
        d = alloc_rows(k, C, ctx.device)
        d.copy_(torch.from_numpy(mine))
        par = rs.encode(d)
        o = alloc_rows(k, C, ctx.device, fill=0)
        dec = PatternDecoder(torch.from_numpy(rs.G).to(ctx.device), [d[i] for i in range(k)] + [par[i] for i in range(n - k)],
                             [o[i] for i in range(k)], e=4)
        if ctx.is_root:
            dec.rows.copy_(torch.tensor(rows, dtype=torch.int32))
        if dist.is_initialized():
            dist.broadcast(dec.rows, 0)
        dec.solve()
        dec.run()
        torch.cuda.synchronize()
        assert int(dec.status.item()) == 0 and np.array_equal(o.cpu().numpy(), mine), "pattern decode mismatch"
        assert sorted(dec.erased.cpu().tolist()) == [2, 4, 7, 9]

    if dist.is_initialized():
        dist.barrier()
    if ctx.is_root:
        print(f"distributed tour OK on {ctx.device.type} with {ctx.world} rank(s) ({ctx.backend})", flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def _spawned(rank: int, world: int, port: int) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    tour(force_pg=False)


def main() -> int:
    if "WORLD_SIZE" in os.environ:  # under torchrun
        tour(force_pg=False)
        return 0
    if torch.cuda.device_count() > 0:  # one GPU, no launcher: a one-rank RCCL group
        tour(force_pg=True)
        return 0
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    torch.multiprocessing.spawn(_spawned, args=(2, port), nprocs=2, join=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
