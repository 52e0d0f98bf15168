#!/usr/bin/env python3
"""Mismatch pattern of one FP4 GEMM against the oracle (debug aid): which output rows / bits /
column phases differ. Usage: GFRS_FP4_KERNEL=ar python scripts/fp4_debug.py K M NCOLS [copy]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpu_rscode_amd.gf import GF256  # noqa: E402
from gpu_rscode_amd.models import alloc_rows  # noqa: E402
from gpu_rscode_amd.ops import GemmPlan  # noqa: E402

k, m, ncols = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
rng = np.random.default_rng(1)
coeff = rng.integers(0, 256, size=(m, k), dtype=np.uint8)
host = rng.integers(0, 256, size=(k, ncols), dtype=np.uint8)
dev = alloc_rows(k, ncols, "cuda")
dev.copy_(torch.from_numpy(host))
out = alloc_rows(m, ncols, "cuda", fill=0x5A)
plan = GemmPlan(dev, out, coeff, engine="mfma")
plan.run()
torch.cuda.synchronize()
got = out.cpu().numpy()
want = GF256.gemm(coeff, host)
bad = got != want
print("rows bad:", [int(r) for r in np.nonzero(bad.any(axis=1))[0]])
print("frac bad per row:", np.round(bad.mean(axis=1), 3).tolist())
cols = np.nonzero(bad.any(axis=0))[0]
print("n bad cols:", len(cols), "first:", cols[:20].tolist())
if len(cols):
    print("col % 128 hist:", np.bincount(cols % 128, minlength=128).tolist())
    x = got ^ want
    print("xor bits hist:", [int(((x >> b) & 1).sum()) for b in range(8)])
    r0 = int(np.nonzero(bad.any(axis=1))[0][0])
    print("row", r0, "got", got[r0, cols[:8]].tolist(), "want", want[r0, cols[:8]].tolist())

# identity probe: out row o should equal input row o; report what it actually matches
if "ident" in sys.argv:
    ident = np.zeros((m, k), dtype=np.uint8)
    for o in range(m):
        ident[o, o] = 1
    out2 = alloc_rows(m, ncols, "cuda", fill=0x5A)
    plan2 = GemmPlan(dev, out2, ident, engine="mfma")
    plan2.run()
    torch.cuda.synchronize()
    g2 = out2.cpu().numpy()
    for o in range(min(m, 8)):
        row = g2[o, :4096]
        best = None
        for r in range(k):
            for sh in range(-40, 41):
                a = host[r, max(0, sh):4096 + min(0, sh)]
                b = row[max(0, -sh):4096 - max(0, sh)]
                frac = float((a == b).mean())
                if best is None or frac > best[0]:
                    best = (frac, r, sh)
        print("out row", o, "best match input row", best[1], "shift", best[2], "frac", round(best[0], 3),
              "sample", row[:8].tolist(), "want", host[o, :8].tolist())
