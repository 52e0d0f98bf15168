#!/usr/bin/env python3
"""What the per-step parity exchange costs the GPU itself (not the links), measured on ONE MI355X.

In the multi-GPU bench (`bench.py --gpus N --comm owners`) every rank sends (N-1)/N of its parity
block to its peers and receives as many bytes from them, asynchronously on RCCL's stream while the
next step computes. On each GPU that is an extra HBM read of the outgoing bytes and an extra HBM
write of the incoming ones, done by copy kernels that share the CUs with the GF-GEMMs. This script
replays exactly that local traffic with no links: after every step, a side stream copies (N-1)/N of
the step's parity into a device buffer (one read + one write per byte, what a GPU's HBM sees under
the all-to-all), double-buffered like the real exchange, and times the bench loop.

The result is the HBM/CU floor of the N-GPU step: the measured multi-GPU step can only be slower
(link time). Together with the busiest-link bytes the bench reports, it splits the N-GPU step into
"GPU side" and "xGMI side".

    python scripts/exchange_cost.py --steps 30            # k=10, n=14, 1 GiB (the headline shape)
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from gpu_rscode_amd import gf  # noqa: E402
from gpu_rscode_amd.models import ReedSolomon  # noqa: E402


class LocalExchange:
    """The ParityExchange interface (sources / start / wait / drain) with the inter-GPU transfer
    replaced by a device-local copy of the bytes an owners all-to-all moves per rank."""

    def __init__(self, sources: list[torch.Tensor], world: int):
        self.sources = sources
        n = sources[0].numel()
        self.nbytes = n - n // world if world > 1 else 0  # bytes that leave (and arrive) per step
        self.recv = torch.empty(max(self.nbytes, 1), dtype=torch.uint8, device=sources[0].device)
        self.stream = torch.cuda.Stream(sources[0].device)
        self.done = [None] * len(sources)

    def start(self, slot: int) -> None:
        if not self.nbytes:
            return
        self.wait(slot)
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            self.recv.copy_(self.sources[slot][: self.nbytes])
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.done[slot] = ev

    def wait(self, slot: int) -> None:
        if self.done[slot] is not None:
            torch.cuda.current_stream().wait_event(self.done[slot])
            self.done[slot] = None

    def drain(self) -> None:
        for s in range(len(self.sources)):
            self.wait(s)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--preset", default="k10n14", choices=sorted(bench.PRESETS))
    ap.add_argument("--worlds", default="1,2,4,8", help="emulated N (fraction (N-1)/N of parity copied)")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    args = bench.parse(["--preset", a.preset, "--steps", str(a.steps), "--warmup", str(a.warmup)])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    k, n = args.k, args.n
    C = (args.bytes + k - 1) // k
    rs = ReedSolomon(k, n)
    pool = bench.erasure_pool(k, n, args.erasures, rs)
    work = bench.GpuWorkload(args, k, n, C, rs.E, gf.GF256.generator(rs.E), pool, 0, dev, 2)
    flats = [work.flat_parity(s) for s in range(len(work.parity))]
    worlds = [int(w) for w in a.worlds.split(",")]
    bytes_per_step = 2 * k * C
    res = {w: [] for w in worlds}
    for _ in range(a.rounds):  # interleaved rounds: clock / thermal drift hits every N alike
        for w in worlds:
            xchg = LocalExchange(flats, w)
            bench.warm(work, xchg, a.warmup)
            el = bench.timed_loop(work, xchg, a.steps, 1, dev, f"exchange_cost/N{w}")
            res[w].append(el / a.steps * 1e3)
    ok = work.verify()
    out = {"preset": a.preset, "steps": a.steps, "verified": bool(ok), "parity_bytes": flats[0].numel(), "per_N": {}}
    base = min(res[worlds[0]])
    for w in worlds:
        ms = min(res[w])
        nbytes = flats[0].numel() - flats[0].numel() // w if w > 1 else 0
        out["per_N"][str(w)] = {
            "ms_per_step_best": round(ms, 4), "ms_per_step_all": [round(x, 4) for x in res[w]],
            "exchange_bytes_per_step": nbytes, "slowdown_vs_no_exchange": round(ms / base, 3),
            "gpu_side_GBps_per_rank": round(bytes_per_step / (ms / 1e3) / 1e9, 1),
        }
    print(json.dumps(out), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
