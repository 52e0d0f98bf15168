#!/usr/bin/env python3
"""Exercise every torch.distributed call the framework issues, over RCCL ("nccl") on GPU tensors.

  python scripts/rccl_probe.py                      # world 1: a forced one-rank RCCL communicator
  torchrun --nproc-per-node 2 scripts/rccl_probe.py --same-device   # 2 ranks sharing cuda:0

Calls: broadcast, all_reduce(MAX/MIN), gather, all_to_all_single (uneven splits, async), and
batch_isend_irecv (to self at world 1, ring neighbours otherwise), each checked for content.
Prints one line per call and "RCCL-PROBE-OK" at the end.
"""
from __future__ import annotations

import argparse
import os
import socket
import sys
import time

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--same-device", action="store_true", help="every rank uses cuda:0")
    ap.add_argument("--bytes", type=int, default=(8 << 20) + 13)
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if a.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    t0 = time.perf_counter()
    if world == 1:
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1, device_id=dev)
    else:
        dist.init_process_group("nccl", device_id=dev)
    print(f"[{rank}] init nccl world={world} dev={dev} {time.perf_counter() - t0:.2f}s", flush=True)

    def ok(name, cond):
        print(f"[{rank}] {name}: {'ok' if cond else 'MISMATCH'}", flush=True)
        if not cond:
            raise SystemExit(1)

    x = torch.arange(40, dtype=torch.int32, device=dev) + (100 if rank == 0 else 0)
    dist.broadcast(x, 0)
    ok("broadcast", torch.equal(x, torch.arange(40, dtype=torch.int32, device=dev) + 100))

    t = torch.tensor([float(rank + 1)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ok("all_reduce MAX", float(t.item()) == world)
    m = torch.tensor([rank], dtype=torch.int32, device=dev)
    dist.all_reduce(m, op=dist.ReduceOp.MIN)
    ok("all_reduce MIN", int(m.item()) == 0)

    g = torch.tensor([rank * 7, rank], dtype=torch.int64, device=dev)
    lst = [torch.empty_like(g) for _ in range(world)] if rank == 0 else None
    dist.gather(g, lst, dst=0)
    if rank == 0:
        ok("gather", all(int(lst[r][0]) == 7 * r and int(lst[r][1]) == r for r in range(world)))

    n = a.bytes
    src = (torch.arange(n, dtype=torch.int64, device=dev) * 13 + rank).remainder(251).to(torch.uint8)
    base, rem = divmod(n, world)
    ins = [base + (1 if r < rem else 0) for r in range(world)]
    mine = ins[rank]
    recv = torch.empty(mine * world, dtype=torch.uint8, device=dev)
    w = dist.all_to_all_single(recv, src, [mine] * world, ins, async_op=True)
    w.wait()
    torch.cuda.synchronize()
    off = sum(ins[:rank])
    want = torch.cat([(torch.arange(off, off + mine, dtype=torch.int64, device=dev) * 13 + r).remainder(251)
                      .to(torch.uint8) for r in range(world)])
    ok("all_to_all_single uneven async", torch.equal(recv, want))

    dst, srcr = (rank + 1) % world, (rank - 1) % world
    got = torch.empty(n, dtype=torch.uint8, device=dev)
    ops = [dist.P2POp(dist.isend, src, dst), dist.P2POp(dist.irecv, got, srcr)]
    for wk in dist.batch_isend_irecv(ops):
        wk.wait()
    torch.cuda.synchronize()
    want = (torch.arange(n, dtype=torch.int64, device=dev) * 13 + srcr).remainder(251).to(torch.uint8)
    ok(f"batch_isend_irecv {rank}->{dst}", torch.equal(got, want))

    # per-row P2P into a pitched destination (the framework's in-place gather pattern)
    rows = torch.empty((3, 4096 + 256), dtype=torch.uint8, device=dev)
    ops = []
    for i in range(3):
        ops.append(dist.P2POp(dist.isend, src[i * 4096:(i + 1) * 4096], dst))
        ops.append(dist.P2POp(dist.irecv, rows[i, :4096], srcr))
    for wk in dist.batch_isend_irecv(ops):
        wk.wait()
    torch.cuda.synchronize()
    ok("per-row batch_isend_irecv into strided rows", all(torch.equal(rows[i, :4096], want[i * 4096:(i + 1) * 4096])
                                                          for i in range(3)))
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        print("RCCL-PROBE-OK", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
