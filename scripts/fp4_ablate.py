#!/usr/bin/env python3
"""Median kernel time of the wide FP4 encode GEMM (k=128, m=32, 1 GiB), one JSON line. Run once
per GFRS_FP4_ABL value (the sk kernel's ablation builds, gf_mfma_fp4.hip) to see which part of
the kernel bounds it: 1 = no epilogue VALU, 2 = no B-expansion masks, 4 = L2-resident input."""
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
    k, m, iters = 128, 32, 20
    C = (1 << 30) // k
    data = alloc_rows(k, C, "cuda")
    fill_random_(flat_rows(data), seed=3)
    coeff = np.random.default_rng(5).integers(1, 256, size=(m, k), dtype=np.uint8)
    out = alloc_rows(m, C, "cuda")
    plan = GemmPlan(data, out, coeff, engine="mfma")
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
    ok = np.array_equal(out[:, :cols].cpu().numpy(), gf.GF256.gemm(coeff, data[:, :cols].cpu().numpy()))
    print(json.dumps({"abl": os.environ.get("GFRS_FP4_ABL", "0"), "median_us": round(float(np.median(ts)), 1),
                      "min_us": round(min(ts), 1), "ok": bool(ok)}), flush=True)


if __name__ == "__main__":
    main()
