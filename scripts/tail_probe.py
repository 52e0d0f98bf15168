#!/usr/bin/env python3
"""Ragged-tail cost of the v_perm GF-GEMM: the same encode (k=10, p=4) and 4-erasure decode with
fused copies on C with and without a < 16-byte tail, median kernel time per shape (one JSON line).
--byte: also time the byte kernel (any alignment; run(vec=0)) and its serial round-3 form
(run(vec=-1)) on the same shapes."""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpu_rscode_amd import ReedSolomon, alloc_rows, flat_rows  # noqa: E402
from gpu_rscode_amd.ops import GemmPlan, fill_random_  # noqa: E402


def med(fn, reps=25):
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
    return round(float(np.median(ts)), 1)


def main():
    rs = ReedSolomon(10, 14)
    res = {}
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    for C in [int(x) for x in (args[0] if args else "107374183,107374176,104858,104848").split(",")]:
        data = alloc_rows(10, C, "cuda")
        fill_random_(flat_rows(data), seed=1)
        par = alloc_rows(4, C, "cuda")
        out = alloc_rows(10, C, "cuda")
        enc = GemmPlan(data, par, rs.E)
        rows = [0, 2, 3, 4, 6, 7, 9, 10, 11, 13]
        surv = [data[r] if r < 10 else par[r - 10] for r in rows]
        erased = [1, 5, 8]
        dm = rs.decode_matrix(rows)[erased]
        copies = [out[r] if r < 10 else None for r in rows]
        dec = GemmPlan(surv, [out[i] for i in erased], dm, copies=copies)
        res[f"C{C}_tail{C % 16}"] = {"enc_us": med(enc.run), "dec_us": med(dec.run)}
        if "--byte" in sys.argv:
            res[f"C{C}_tail{C % 16}"].update(byte_enc_us=med(lambda: enc.run(vec=0), 5),
                                             byte_dec_us=med(lambda: dec.run(vec=0), 5),
                                             serial_byte_enc_us=med(lambda: enc.run(vec=-1), 5),
                                             serial_byte_dec_us=med(lambda: dec.run(vec=-1), 5))
            out.zero_()
            dec.run(vec=0)
            torch.cuda.synchronize()
            assert torch.equal(out, data), "byte kernel decode mismatch"
        torch.cuda.synchronize()
        assert torch.equal(out, data)
        del data, par, out, enc, dec, surv, copies
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
