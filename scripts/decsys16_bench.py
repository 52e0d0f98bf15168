#!/usr/bin/env python3
"""GF(2^16) decode-plan solve: the host path (gfrs::gf16w::decode_rows, the e x e systematic solve
in C++) against the device (gf_decode16.hip: one workgroup when the e x (e + k) system fits its
LDS, else the blocked multi-workgroup solve), for wide codes (k = 2000 / e = 100,
k = 4000 / e = 500). The device time is the whole plan build on an idle GPU (pattern check, solve,
tables); the device plan is checked bit-exactly against the host rows. Prints one JSON object."""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpu_rscode_amd import ReedSolomon  # noqa: E402
from gpu_rscode_amd._native import cpu, hip  # noqa: E402
from gpu_rscode_amd.models import alloc_rows  # noqa: E402
from gpu_rscode_amd.ops.gemm import Gemm16Plan  # noqa: E402
from gpu_rscode_amd.ops.inverse import decode_system16_into_plan  # noqa: E402


def case(k, n, e, reps=5):
    rs = ReedSolomon(k, n, field="gf65536", matrix="cauchy")
    rng = np.random.default_rng(k + e)
    erased = sorted(rng.choice(k, size=e, replace=False).tolist())
    rows = [r for r in range(k) if r not in erased] + sorted(rng.choice(range(k, n), size=e, replace=False).tolist())
    gb = np.ascontiguousarray(rs.G, dtype="<u2").tobytes()
    host = []
    for _ in range(3):
        t = time.perf_counter()
        raw = cpu().gf16_decode_rows(gb, k, rows, erased)
        host.append((time.perf_counter() - t) * 1e3)
    want = np.frombuffer(raw, dtype="<u2").reshape(e, k)
    g = torch.from_numpy(np.ascontiguousarray(rs.G, dtype="<u2").view(np.int16)).cuda()
    plan = Gemm16Plan(alloc_rows(k, 64, "cuda"), alloc_rows(e, 64, "cuda"), device_tables=True, engine="valu16")
    rows_d = torch.tensor(rows, dtype=torch.int32, device="cuda")
    er_d = torch.zeros(e, dtype=torch.int32, device="cuda")
    dm = torch.zeros((e, k), dtype=torch.int16, device="cuda")
    st = decode_system16_into_plan(g, rows_d, er_d, plan, dm=dm)  # warm (code objects, workspace)
    torch.cuda.synchronize()
    ok = int(st.item()) == 0 and er_d.tolist() == erased and np.array_equal(dm.cpu().numpy().view("<u2"), want)
    dev = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        decode_system16_into_plan(g, rows_d, er_d, plan, status=st)
        b.record()
        torch.cuda.synchronize()
        dev.append(a.elapsed_time(b))
    return {"k": k, "n": n, "e": e, "system_bytes": 2 * e * (e + k),
            "device_path": "one-workgroup" if hip().decode_system16_supported(n, k, e) else "blocked",
            "host_ms_median": round(float(np.median(host)), 3), "device_ms_median": round(float(np.median(dev)), 3),
            "device_ms_min": round(min(dev), 3), "bit_exact_vs_host": bool(ok)}


def main():
    shapes = [(300, 340, 40), (2000, 2100, 100), (4000, 4500, 500), (1000, 2000, 1000)]
    if len(sys.argv) > 1:
        shapes = [tuple(int(x) for x in s.split(":")) for s in sys.argv[1].split(",")]
    print(json.dumps({"cases": [case(*s) for s in shapes]}), flush=True)


if __name__ == "__main__":
    main()
