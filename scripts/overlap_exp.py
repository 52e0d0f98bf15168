#!/usr/bin/env python3
"""Experiment: wide-stripe decode as (plain FP4 GEMM) + (survivor copy on a side stream) vs the
fused-copy FP4 kernel. The wide GEMM is matrix-core bound (~1.3 TB/s of HBM), so a copy kernel that
co-resides on the CUs' leftover registers could use the idle HBM bandwidth.

    python scripts/overlap_exp.py --k 128 --m 26 --copies 102
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


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = []
    for _ in range(iters):
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        best.append(s.elapsed_time(e) * 1e3)
    return round(float(np.median(best)), 1), round(float(min(best)), 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--m", type=int, default=26)
    ap.add_argument("--copies", type=int, default=102)
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    C = (a.bytes + a.k - 1) // a.k
    data = alloc_rows(a.k, C, "cuda")
    fill_random_(flat_rows(data), seed=1)
    out = alloc_rows(a.m, C, "cuda")
    dst = alloc_rows(a.copies, C, "cuda")
    coeff = np.random.default_rng(0).integers(1, 256, size=(a.m, a.k), dtype=np.uint8)
    copies = [dst[j] if j < a.copies else None for j in range(a.k)]
    fused = GemmPlan(data, out, coeff, copies=copies, engine="mfma")
    plain = GemmPlan(data, out, coeff, engine="mfma")
    main_s = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    src = data[: a.copies]
    dsts = dst[: a.copies]

    def copy_only():
        dsts.copy_(src)

    def both(copy_first):
        def run():
            side.wait_stream(main_s)
            if copy_first:
                with torch.cuda.stream(side):
                    dsts.copy_(src)
                plain.run()
            else:
                plain.run()
                with torch.cuda.stream(side):
                    dsts.copy_(src)
            main_s.wait_stream(side)
        return run

    res = {}
    for mode in ("fused", "split", "split_first"):
        os.environ["GFRS_FP4_COPY"] = mode
        dst.zero_()
        res[f"decode_{mode}_us"] = timeit(fused.run, a.iters)
        torch.cuda.synchronize()
        res[f"decode_{mode}_copy_ok"] = bool(torch.equal(dsts, src))
    os.environ["GFRS_FP4_COPY"] = "split"
    res.update({
        "fused_us": timeit(fused.run, a.iters),
        "plain_us": timeit(plain.run, a.iters),
        "copy_us": timeit(copy_only, a.iters),
        "plain_then_copy_side_us": timeit(both(False), a.iters),
        "copy_side_then_plain_us": timeit(both(True), a.iters),
    })
    torch.cuda.synchronize()
    ok = torch.equal(dsts, src)
    fused.run()
    o1 = out.clone()
    plain.run()
    ok = ok and torch.equal(o1, out)
    res["ok"] = bool(ok)
    res["args"] = vars(a)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
