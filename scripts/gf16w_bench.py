#!/usr/bin/env python3
"""GF(2^16) kernel timings on one MI355X next to the GF(2^8) kernel on the same stripe shape.

For each (k, n): 1 GiB of native bytes in HBM (device-generated), then
  encode  parity[p] = E . data[k]                         (GF(2^16): csrc/kernels/gf_gemm16.hip)
  decode  the first min(k, p) natives erased; k survivors -> all k natives, rebuilt ones computed
          and surviving ones copied in the same pass (fused copy)
each timed with HIP events over --reps launches (median), and the same two ops in GF(2^8)
(csrc/kernels/gf_gemm.hip) when n <= 256. Bytes moved per op = rows read + rows written; GB/s is
that over the kernel time. Prints one JSON object.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpu_rscode_amd import ReedSolomon, alloc_rows, flat_rows  # noqa: E402
from gpu_rscode_amd.ops import fill_random_  # noqa: E402


def _time(fn, reps: int) -> float:
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


def case(k: int, n: int, nbytes: int, field: str, reps: int) -> dict:
    p = n - k
    C = (nbytes + k - 1) // k
    if field == "gf65536":
        C += C % 2
    rs = ReedSolomon(k, n, field=field, matrix="cauchy" if n > 256 else "vandermonde")
    data = alloc_rows(k, C, "cuda")
    fill_random_(flat_rows(data), seed=k)
    par = alloc_rows(p, C, "cuda")
    enc_ms = _time(lambda: rs.encode(data, par), reps)
    e = min(k, p)
    rows = list(range(e, k)) + list(range(k, k + e))
    stripe = [data[r] if r < k else par[r - k] for r in rows]
    out = alloc_rows(k, C, "cuda")
    dec_ms = _time(lambda: rs.decode(stripe, rows, out=out), reps)
    ok = bool(torch.equal(out, data))
    enc_bytes, dec_bytes = (k + p) * C, 2 * k * C
    return {"field": field, "k": k, "n": n, "chunk_bytes": C, "encode_ms": round(enc_ms, 4),
            "decode_ms": round(dec_ms, 4), "erased": e,
            "encode_GBps_traffic": round(enc_bytes / enc_ms / 1e6, 1),
            "decode_GBps_traffic": round(dec_bytes / dec_ms / 1e6, 1),
            "encode_decode_GBps": round(2 * k * C / (enc_ms + dec_ms) / 1e6, 1), "decode_verified": ok}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--shapes", default="10:14,300:340")
    a = ap.parse_args()
    res = []
    for s in a.shapes.split(","):
        k, n = (int(v) for v in s.split(":"))
        res.append(case(k, n, a.bytes, "gf65536", a.reps))
        if n <= 256:
            res.append(case(k, n, a.bytes, "gf256", a.reps))
        torch.cuda.empty_cache()
    print(json.dumps({"bytes": a.bytes, "reps": a.reps, "results": res}))
    return 0 if all(r["decode_verified"] for r in res) else 1


if __name__ == "__main__":
    sys.exit(main())
