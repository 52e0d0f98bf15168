#!/usr/bin/env python3
"""Kernel micro-benchmark: GF-GEMM variants on the BASELINE shapes, interleaved rounds in one
process (cdna_hip_programming.md §5.4 rule 24), plus an HBM copy roofline and the inverse kernel.

Writes JSON to stdout (and --out). Traffic model: every input row read once, every output and
fused-copy row written once.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpu_rscode_amd import gf  # noqa: E402
from gpu_rscode_amd.models import alloc_rows, flat_rows  # noqa: E402
from gpu_rscode_amd.ops import GemmPlan, fill_random_, gf_invert  # noqa: E402

VARIANTS = [None, (1, 1, False), (1, 2, False), (1, 4, False), (1, 2, True), (1, 4, True), (2, 1, False),
            (2, 2, False), (2, 2, True), "mfma", "mfma_mg4", "mfma_mg2", "mfma_i8", "lut"]


def timed(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def make_case(name, k, m, ncopy, total_bytes):
    C = (total_bytes + k - 1) // k
    data = alloc_rows(k, C, "cuda")
    fill_random_(flat_rows(data), seed=k)
    out = alloc_rows(m, C, "cuda")
    copies = None
    if ncopy:
        dst = alloc_rows(ncopy, C, "cuda")
        copies = [dst[j] if j < ncopy else None for j in range(k)]
    coeff = np.random.default_rng(k + m).integers(1, 256, size=(m, k), dtype=np.uint8)
    plan = GemmPlan(data, out, coeff, copies=copies, engine="valu")
    mplan = {"mfma": GemmPlan(data, out, coeff, copies=copies, engine="mfma"),
             "mfma_mg4": GemmPlan(data, out, coeff, copies=copies, engine="mfma", mfma_mg=4),
             "mfma_mg2": GemmPlan(data, out, coeff, copies=copies, engine="mfma", mfma_mg=2)}
    if not ncopy:
        mplan["mfma_i8"] = GemmPlan(data, out, coeff, engine="mfma_i8")
    mplan["lut"] = GemmPlan(data, out, coeff, copies=copies, engine="lut")  # LDS nibble tables (ablation)
    traffic = (k + m + ncopy) * C
    return {"name": name, "k": k, "m": m, "copies": ncopy, "C": C, "plan": plan, "mplan": mplan,
            "traffic": traffic, "keep": (data, out, copies)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default=None)
    ap.add_argument("--cases", default=None, help="comma-separated case names (default: all)")
    ap.add_argument("--variants", default=None,
                    help="semicolon-separated variants, e.g. 'None;1,2,1;1,16,1;mfma' (default: all)")
    a = ap.parse_args()

    res = {"device": torch.cuda.get_device_name(0), "cases": {}}
    # HBM roofline: device-to-device copy of the same volume
    src = torch.empty(a.bytes, dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)
    us = min(timed(lambda: dst.copy_(src), a.reps) for _ in range(3))
    res["copy_roofline_TBps"] = round(2 * a.bytes / us / 1e6, 3)
    del src, dst

    specs = [("enc_k10_p4", 10, 4, 0), ("dec_k10_e4_copy6", 10, 4, 6), ("enc_k4_p2", 4, 2, 0), ("enc_k16_p4", 16, 4, 0),
             ("enc_k128_p32", 128, 32, 0), ("dec_k10_e1_copy9", 10, 1, 9), ("dec_k128_e32_copy96", 128, 32, 96),
             ("dec_k16_e4_copy12", 16, 4, 12)]
    keep = set(a.cases.split(",")) if a.cases else None
    cases = (make_case(nm, k, m, nc, a.bytes) for nm, k, m, nc in specs if keep is None or nm in keep)
    variants = VARIANTS
    if a.variants:
        variants = []
        for tok in a.variants.split(";"):
            if tok == "None":
                variants.append(None)
            elif tok.startswith("mfma") or tok == "lut":
                variants.append(tok)
            else:
                v, pf, nt = (int(x) for x in tok.split(","))
                variants.append((v, pf, bool(nt)))
    for c in cases:
        times = {str(v): [] for v in variants}
        for _ in range(a.rounds):
            for v in variants:
                if isinstance(v, str):
                    if v not in c["mplan"]:
                        continue
                    pl = c["mplan"][v]
                    pl.run()
                    times[str(v)].append(timed(lambda: pl.run(), a.reps))
                    continue
                kw = {} if v is None else dict(vec=v[0], pf=v[1], nt=v[2])
                try:
                    c["plan"].run(**kw)  # warm
                except RuntimeError as e:
                    raise RuntimeError(f"{c['name']} variant {v}: {e}") from e
                times[str(v)].append(timed(lambda: c["plan"].run(**kw), a.reps))
        out = {}
        for v, ts in times.items():
            if not ts:
                continue
            med = float(np.median(ts))
            out[v] = {"us_median": round(med, 2), "us_min": round(min(ts), 2),
                      "TBps": round(c["traffic"] / med / 1e6, 3),
                      "input_GBps": round(c["k"] * c["C"] / med / 1e3, 1)}
        res["cases"][c["name"]] = {"k": c["k"], "m": c["m"], "copies": c["copies"], "C": c["C"], "variants": out}
        del c["plan"], c["keep"], c["mplan"]
        torch.cuda.empty_cache()

    for n in (10, 16, 128, 255):
        g = np.random.default_rng(n)
        while True:
            m = g.integers(0, 256, size=(n, n), dtype=np.uint8)
            if gf.GF256.is_invertible(m):
                break
        t = torch.from_numpy(m).cuda()
        gf_invert(t)
        res[f"invert_n{n}_us"] = round(min(timed(lambda: gf_invert(t, check=False), 20) for _ in range(3)), 2)

    js = json.dumps(res, indent=1)
    print(js)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js)


if __name__ == "__main__":
    main()
