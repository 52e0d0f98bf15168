#!/usr/bin/env python3
"""Bit-exact check of the FP4 GEMM on k = 128 shapes under whatever GFRS_TUNE the caller sets (e.g.
fp4=tm to force the tile-major form): 5-8 tiles with fused copies, and 5-8 tiles plain with
uniform-stride and with scattered input rows; several chunk counts per persistent block (odd and
even) and a ragged column tail. Prints one line per case, exits non-zero on the first mismatch."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpu_rscode_amd.gf import GF256
from gpu_rscode_amd.models import alloc_rows
from gpu_rscode_amd.ops import GemmPlan


def main() -> int:
    k = 128
    cases = [(m, "copies") for m in (20, 21, 22, 24, 26, 28, 29, 32)]
    cases += [(m, kind) for m in (20, 24, 28, 29, 32) for kind in ("uniform", "scattered")]
    for m, kind in cases:
        for ncols in (256 * 256 * 3 + 77, 256 * 256 * 6 + 2, 256 * 1000 + 130):
            g = np.random.default_rng(m * 7 + ncols)
            host = g.integers(0, 256, size=(k, ncols), dtype=np.uint8)
            coeff = g.integers(0, 256, size=(m, k), dtype=np.uint8)
            dev = alloc_rows(k, ncols, "cuda")
            dev.copy_(torch.from_numpy(host))
            rows = [dev[j] for j in range(k)]
            if kind == "scattered":  # the same rows in another order: no common stride
                perm = g.permutation(k)
                rows = [rows[j] for j in perm]
                host = host[perm]
            cdst = alloc_rows(k, ncols, "cuda", fill=0) if kind == "copies" else None
            copies = [cdst[j] if j % 5 else None for j in range(k)] if kind == "copies" else None
            out = alloc_rows(m, ncols, "cuda", fill=0)
            plan = GemmPlan(rows, out, coeff, copies=copies, engine="mfma")
            plan.run()
            torch.cuda.synchronize()
            ok = np.array_equal(out.cpu().numpy(), GF256.gemm(coeff, host))
            ok_c = True
            if cdst is not None:
                c = cdst.cpu().numpy()
                ok_c = all(np.array_equal(c[j], host[j]) if j % 5 else not c[j].any() for j in range(k))
            print(f"m={m} {kind} ncols={ncols} form={getattr(plan, 'fp4_form', None)} gemm={ok} copies={ok_c}",
                  flush=True)
            if not (ok and ok_c):
                return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
