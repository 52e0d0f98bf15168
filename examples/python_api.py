#!/usr/bin/env python3
"""Python API tour: device-resident encode, erasure decode with the on-device inverse, in-place
repair, batched small objects, the CPU fallback, the wide-stripe matrix-core engine and GF(2^16)
codes past 256 chunks.

    python examples/python_api.py            # on an MI355X box (falls back to CPU tensors otherwise)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from gpu_rscode_amd import ReedSolomon, alloc_rows  # noqa: E402
from gpu_rscode_amd.gf import GF256, field  # noqa: E402


def main():
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    k, n, C = 10, 14, 1_000_003
    rs = ReedSolomon(k, n)  # the reference's Vandermonde; matrix="cauchy" gives an MDS code
    host = np.random.default_rng(0).integers(0, 256, size=(k, C), dtype=np.uint8)
    data = alloc_rows(k, C, dev)
    data.copy_(torch.from_numpy(host))
    parity = rs.encode(data)
    stripe = [data[i] for i in range(k)] + [parity[i] for i in range(n - k)]

    # lose chunks 1, 4, 11, 12 (natives and parity); decode from the k survivors
    rows = [r for r in range(n) if r not in (1, 4, 11, 12)]
    out = rs.decode([stripe[r] for r in rows], rows, device_invert=(dev == "cuda"))
    assert np.array_equal(out.cpu().numpy(), host)

    # in-place repair of a whole stripe (natives and parity rebuilt in one GEMM)
    full = alloc_rows(n, C, dev)
    full[:k].copy_(data)
    full[k:].copy_(parity)
    want = full.clone()
    full[[0, 5, 13]] = 0
    rs.reconstruct(full, [0, 5, 13])
    assert torch.equal(full, want)

    # many small objects: one launch for B stripes
    if dev == "cuda":
        objs = torch.randint(0, 256, (64, k, 4096), dtype=torch.uint8, device=dev)
        par = rs.encode_batch(objs)
        assert np.array_equal(par[7].cpu().numpy(), GF256.gemm(rs.E, objs[7].cpu().numpy()))

        # wide stripes pick the FP4 matrix-core kernel automatically
        wide = ReedSolomon(128, 160, matrix="cauchy")
        wd = alloc_rows(128, 1 << 20, dev)
        wd.random_(0, 256)
        wp = wide.encode(wd)
        torch.cuda.synchronize()
        assert np.array_equal(wp[:, :4096].cpu().numpy(), GF256.gemm(wide.E, wd[:, :4096].cpu().numpy()))
    # GF(2^16) (the reference's w = 16 field): 16-bit symbols, so n may exceed 256
    big = ReedSolomon(300, 340, field="gf65536", matrix="cauchy")
    bd = alloc_rows(300, 2 * 4099, dev)  # even byte rows: little-endian 16-bit symbols
    bd.copy_(torch.from_numpy(np.random.default_rng(3).integers(0, 256, size=(300, 2 * 4099), dtype=np.uint8)))
    bp = big.encode(bd)
    sym = bd.cpu().numpy().view("<u2")
    assert np.array_equal(bp.cpu().numpy().view("<u2"), field(16).gemm(big.E, sym))
    lost = set(range(0, 300, 8)) | {300, 333}  # 38 natives and 2 parity chunks
    keep = [r for r in range(340) if r not in lost][:300]
    bstripe = [bd[i] for i in range(300)] + [bp[i] for i in range(40)]
    assert torch.equal(big.decode([bstripe[r] for r in keep], keep), bd)
    print(f"python API tour OK on {dev}")


if __name__ == "__main__":
    main()
