#!/usr/bin/env python3
"""Where the FP4 matrix-core engine starts to beat the v_perm engine, by row length.

For wide codes (k, m) and chunk sizes C, one GemmPlan per engine on the same rows, event-timed
(median of --reps launches after a warm-up), encode and a decode-shaped GEMM with fused copies
(copies of the first k - m inputs). Prints one JSON line per point; every output is checked
against the other engine's.

  python scripts/engine_cross.py [--shapes 128:32,64:16,32:8] [--cols 8192,65536,524288,8388608]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpu_rscode_amd.models import alloc_rows, flat_rows  # noqa: E402
from gpu_rscode_amd.ops import GemmPlan, fill_random_  # noqa: E402


def timed(fn, reps: int) -> float:
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return float(np.median(ts))


def point(k: int, m: int, C: int, reps: int, copies: bool) -> dict:
    data = alloc_rows(k, C, "cuda")
    fill_random_(flat_rows(data), seed=k + m)
    coeff = np.random.default_rng(k * m).integers(1, 256, size=(m, k), dtype=np.uint8)
    res = {"k": k, "m": m, "C": C, "copies": copies}
    outs = {}
    for eng in ("valu", "mfma"):
        out = alloc_rows(m, C, "cuda", fill=0)
        cp = alloc_rows(k, C, "cuda", fill=0) if copies else None
        cps = [cp[j] if j < k - m else None for j in range(k)] if copies else None
        plan = GemmPlan(data, out, coeff, copies=cps, engine=eng)
        res[f"{eng}_us"] = round(timed(plan.run, reps), 2)
        outs[eng] = out
    torch.cuda.synchronize()
    res["agree"] = bool(torch.equal(outs["valu"], outs["mfma"]))
    res["mfma_speedup"] = round(res["valu_us"] / res["mfma_us"], 3)
    return res


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--shapes", default="128:32,64:16,32:8")
    ap.add_argument("--cols", default="8192,65536,524288,8388608")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    ok = True
    for s in a.shapes.split(","):
        k, m = (int(v) for v in s.split(":"))
        for C in (int(c) for c in a.cols.split(",")):
            for copies in (False, True):
                r = point(k, m, C, a.reps, copies)
                ok = ok and r["agree"]
                print(json.dumps(r), flush=True)
                torch.cuda.empty_cache()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
