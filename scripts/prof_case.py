#!/usr/bin/env python3
"""Run one GF-GEMM case repeatedly (for rocprofv3 --pmc / --kernel-trace on a single kernel).

    rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU ... -- python3 scripts/prof_case.py --k 128 --m 32 --engine valu
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpu_rscode_amd.models import alloc_rows, flat_rows  # noqa: E402
from gpu_rscode_amd.ops import GemmPlan, fill_random_  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--copies", type=int, default=0)
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--engine", default="valu")
    ap.add_argument("--vec", type=int, default=None)
    ap.add_argument("--pf", type=int, default=2)
    ap.add_argument("--nt", type=int, default=1)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--field", type=int, default=8, choices=[8, 16], help="16: a GF(2^16) plan (Gemm16Plan)")
    a = ap.parse_args()
    C = (a.bytes + a.k - 1) // a.k
    C += C % 2 if a.field == 16 else 0
    data = alloc_rows(a.k, C, "cuda")
    fill_random_(flat_rows(data), seed=1)
    out = alloc_rows(a.m, C, "cuda")
    copies = None
    if a.copies:
        dst = alloc_rows(a.copies, C, "cuda")
        copies = [dst[j] if j < a.copies else None for j in range(a.k)]
    if a.field == 16:
        from gpu_rscode_amd.ops import Gemm16Plan

        coeff = np.random.default_rng(0).integers(1, 65536, size=(a.m, a.k))
        plan = Gemm16Plan(data, out, coeff, copies=copies, engine=a.engine)
        kw = {}
    else:
        coeff = np.random.default_rng(0).integers(1, 256, size=(a.m, a.k), dtype=np.uint8)
        plan = GemmPlan(data, out, coeff, copies=copies, engine=a.engine)
        kw = {} if a.vec is None else dict(vec=a.vec, pf=a.pf, nt=bool(a.nt))
    for _ in range(a.iters):
        plan.run(**kw)
    torch.cuda.synchronize()
    print("done", a)


if __name__ == "__main__":
    main()
