#!/usr/bin/env python3
"""Host pipeline sweep (csrc/runtime/pipeline.cpp): pinned host rows -> H2D -> GF-GEMM -> D2H for
k=10 -> m rows of a 1 GiB stripe, over -s streams, copy-in stream split, 2-D copies and slice width.
One JSON line per configuration (best of `--reps` calls after one warm call)."""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpu_rscode_amd._native import hip  # noqa: E402
from gpu_rscode_amd.gf import GF256  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--streams", default="1,2,4")
    ap.add_argument("--split", default="0,1")
    ap.add_argument("--rect", default="0,1")
    ap.add_argument("--slices", default=f"{16 << 20},{32 << 20},{64 << 20}")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cold", default=None,
                    help="comma list of hipHostMalloc flags (ints): per configuration and flag, fresh pinned "
                         "buffers written by the CPU, first (cold) call timed, then warm calls")
    a = ap.parse_args()
    if a.cold is not None:
        return cold(a)
    k, m = a.k, a.m
    C = (a.bytes + k - 1) // k
    host = torch.empty((k, C), dtype=torch.uint8, pin_memory=True)
    host.copy_(torch.randint(0, 256, (k, C), dtype=torch.uint8, device="cuda"))
    out = torch.empty((m, C), dtype=torch.uint8, pin_memory=True)
    e = GF256.vandermonde_ref(k, m)
    ins = [host[j].data_ptr() for j in range(k)]
    outs = [out[i].data_ptr() for i in range(m)]
    h = hip()
    for S, split, rect, sl in itertools.product(*(map(int, x.split(",")) for x in (a.streams, a.split, a.rect,
                                                                                      a.slices))):
        def run():
            return h.gemm_host([0], ins, outs, e.tobytes(), C, S, sl, 0, False, split, bool(rect))["devices"][0]

        run()
        best = min((run() for _ in range(a.reps)), key=lambda d: d["ms_total"])
        rec = dict(streams=S, split=split, rect=rect, slice=sl, ms_total=round(best["ms_total"], 3),
                   ms_stream=round(best["ms_stream"], 3), slices=best["slices"], lanes=best["lanes"],
                   h2d_GBps=round(k * C / best["ms_stream"] / 1e6, 2))
        print(json.dumps(rec), flush=True)
    cols = min(C, 1 << 16)
    ok = np.array_equal(out[:, :cols].numpy(), GF256.gemm(e, host[:, :cols].numpy()))
    print(json.dumps({"verified": bool(ok)}))
    return 0 if ok else 1


def cold(a) -> int:
    """First-call cost on fresh pinned buffers (what a CLI encode of a just-read file pays)."""
    import ctypes

    k, m = a.k, a.m
    C = (a.bytes + k - 1) // k
    h = hip()
    e = GF256.vandermonde_ref(k, m)
    ok = True
    for flags in map(int, a.cold.split(",")):
        for S, split, rect, sl in itertools.product(*(map(int, x.split(",")) for x in (a.streams, a.split, a.rect,
                                                                                          a.slices))):
            pin = h.host_alloc(k * C, flags)
            pout = h.host_alloc(m * C, flags)
            src = np.frombuffer((ctypes.c_uint8 * (k * C)).from_address(pin), dtype=np.uint8)
            src[:] = 7  # CPU first touch, like read() into the buffer
            ins = [pin + j * C for j in range(k)]
            outs = [pout + i * C for i in range(m)]
            h.prepare_pipeline([0], k, m, C, S, sl)

            def run():
                return h.gemm_host([0], ins, outs, e.tobytes(), C, S, sl, 0, False, split, bool(rect))["devices"][0]

            first = run()
            warm = min((run() for _ in range(a.reps)), key=lambda d: d["ms_total"])
            dst = np.frombuffer((ctypes.c_uint8 * (m * C)).from_address(pout), dtype=np.uint8)
            want = GF256.gemm(e, np.full((k, 4096), 7, dtype=np.uint8))
            ok = ok and all(np.array_equal(dst[i * C:i * C + 4096], want[i]) for i in range(m))
            print(json.dumps(dict(flags=hex(flags), streams=S, split=split, rect=rect, slice=sl,
                                  cold_ms=round(first["ms_total"], 3), warm_ms=round(warm["ms_total"], 3))), flush=True)
            h.host_free(pin)
            h.host_free(pout)
    print(json.dumps({"verified": bool(ok)}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
