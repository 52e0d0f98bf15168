#!/usr/bin/env python3
"""Median kernel time of wide FP4 GEMM shapes (k=128; m rebuilt rows; optional fused copies), one
JSON line, with the form the router ran. Run once per GFRS_TUNE=fp4=... setting (v1 / ar / tm) to A/B
the FP4 kernel forms."""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpu_rscode_amd import gf  # noqa: E402
from gpu_rscode_amd.models import alloc_rows, flat_rows  # noqa: E402
from gpu_rscode_amd.ops import GemmPlan, fill_random_  # noqa: E402


def main():
    k, C, iters = 128, (1 << 30) // 128, 15
    data = alloc_rows(k, C, "cuda")
    fill_random_(flat_rows(data), seed=3)
    dst = alloc_rows(k, C, "cuda")
    res = {"env": {"GFRS_TUNE": os.environ.get("GFRS_TUNE")}}
    rng = np.random.default_rng(5)
    ms = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [20, 24, 28, 32]
    if "--scattered" in sys.argv:  # inputs as separate allocations (the row-pointer-table kernels)
        rows = [data[j].clone() for j in range(k)]
        del data
        torch.cuda.empty_cache()
        data = rows
    for m in ms:
        coeff = rng.integers(1, 256, size=(m, k), dtype=np.uint8)
        out = alloc_rows(m, C, "cuda")
        for ncopy in (0, 128 - m):
            copies = [dst[j] if j < ncopy else None for j in range(k)] if ncopy else None
            plan = GemmPlan(data, out, coeff, copies=copies, engine="mfma")
            plan.run()
            torch.cuda.synchronize()
            ts = []
            for _ in range(iters):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                plan.run()
                e.record()
                torch.cuda.synchronize()
                ts.append(s.elapsed_time(e) * 1e3)
            cols = 1 << 16
            src = torch.stack([r[:cols] for r in data]) if isinstance(data, list) else data[:, :cols]
            ok = np.array_equal(out[:, :cols].cpu().numpy(), gf.GF256.gemm(coeff, src.cpu().numpy()))
            if ncopy:
                ok = ok and all(torch.equal(dst[j], data[j]) for j in range(ncopy))
            from gpu_rscode_amd._native import hip
            res[f"m{m}_copies{ncopy}"] = {"median_us": round(float(np.median(ts)), 1), "min_us": round(min(ts), 1),
                                          "ok": bool(ok), "form": hip().fp4_route(k, m, bool(ncopy), 8)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
