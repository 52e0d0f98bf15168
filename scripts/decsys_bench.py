#!/usr/bin/env python3
"""Time the on-device decode-system solve (gf_decode_system_kernel) alone, on an idle GPU, for the
BASELINE decode shapes: k=10 with 4 erasures and k=128 with 32 erasures (plus the bit-matrix
rebuild the matrix-core engine adds). Prints one JSON object."""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpu_rscode_amd import gf  # noqa: E402
from gpu_rscode_amd.models import alloc_rows  # noqa: E402
from gpu_rscode_amd.ops import GemmPlan, decode_system_into_plan  # noqa: E402


def case(k, n, e, matrix, reps=50):
    g_host = gf.GF256.generator(gf.GF256.encoding_matrix(matrix, k, n - k))
    g = torch.from_numpy(np.ascontiguousarray(g_host)).cuda()
    erased = list(range(0, 2 * e, 2))[:e]
    rows = [r for r in range(n) if r not in erased][:k]
    C = 1 << 16
    ins = alloc_rows(k, C, "cuda")
    out = alloc_rows(e, C, "cuda")
    res = {}
    for engine in ("valu", "mfma"):
        plan = GemmPlan([ins[i] for i in range(k)], [out[i] for i in range(e)], device_tables=True, engine=engine)
        rows_d = torch.tensor(rows, dtype=torch.int32, device="cuda")
        er_d = torch.tensor(erased, dtype=torch.int32, device="cuda")
        st = decode_system_into_plan(g, rows_d, er_d, plan)
        torch.cuda.synchronize()
        assert int(st.item()) == 0
        s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            decode_system_into_plan(g, rows_d, er_d, plan, status=st)
        t.record()
        t.synchronize()
        res[plan.engine] = round(s.elapsed_time(t) / reps * 1e3, 2)
    return res


def main():
    out = {"k10_e4_us": case(10, 14, 4, "vandermonde"), "k128_e32_us": case(128, 160, 32, "cauchy")}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
