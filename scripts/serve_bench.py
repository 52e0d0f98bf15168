#!/usr/bin/env python3
"""Small-object serving throughput: many RS(10,14) objects per launch (the batched descriptor,
grid.y = object) against one launch per object, and the batched encode + decode replayed from a
captured hipGraph. Device-resident objects; one JSON line per (object size, batch) point.

  python scripts/serve_bench.py [--sizes 65536,262144,1048576,4194304] [--batches 1,16,256] [--out F]

Per point: encode (parity of every object) and decode (3 natives + 1 parity lost on every object,
erased natives rebuilt and surviving natives copied in the same pass) — each as one batched launch,
as a loop of per-object launches, and both batched launches from one graph replay. Verified
against the numpy oracle on the first and last object.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpu_rscode_amd import ReedSolomon, gf  # noqa: E402
from gpu_rscode_amd.ops import fill_random_  # noqa: E402

PITCH = 256


def batch_rows(B: int, rows: int, C: int, dev) -> torch.Tensor:
    pitch = max(PITCH, (C + PITCH - 1) // PITCH * PITCH)
    base = torch.empty(B * rows * pitch, dtype=torch.uint8, device=dev)
    return base.as_strided((B, rows, C), (rows * pitch, pitch, 1)), base


def timed(fn, reps: int) -> float:
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
    return float(np.median(ts))


def point(S: int, B: int, reps: int, k: int = 10, n: int = 14, erase: int = 0, field: int = 8) -> dict:
    p = n - k
    C = (S + k - 1) // k
    if field == 16:
        C += C % 2  # whole 16-bit symbols
    dev = torch.device("cuda", 0)
    rs = ReedSolomon(k, n, **({"field": "gf65536", "matrix": "cauchy"} if field == 16 else {}))
    data, dbase = batch_rows(B, k, C, dev)
    fill_random_(dbase, seed=S + B)
    parity, _ = batch_rows(B, p, C, dev)
    if erase:  # natives 0, 2, 4, ... lost, rebuilt from the first `erase` parity rows
        lost = list(range(0, 2 * erase, 2))[:erase]
        rows = [r for r in range(k) if r not in lost] + list(range(k, k + len(lost)))
    elif (k, n) == (10, 14):
        rows = [0, 2, 3, 4, 6, 7, 9, 10, 11, 13]  # natives 1, 5, 8 and parity 12 lost on every object
    else:  # up to three natives and the first parity lost
        lost = sorted({1, k // 2, k - 2})[:max(1, min(3, p - 1))] + ([k] if p > 1 else [])
        rows = [r for r in range(n) if r not in lost][:k]
    surv, _ = batch_rows(B, k, C, dev)
    out, _ = batch_rows(B, k, C, dev)

    def enc_batched():
        rs.encode_batch(data, parity)

    def dec_batched():
        rs.decode_batch(surv, rows, out)

    def enc_loop():
        for b in range(B):
            rs.encode(data[b], parity[b])

    def dec_loop():
        for b in range(B):
            rs.decode(surv[b], rows, out[b])

    enc_batched()
    for j, r in enumerate(rows):  # the survivors as the decode reads them
        surv[:, j].copy_(data[:, r] if r < k else parity[:, r - k])
    torch.cuda.synchronize()
    res = {"object_bytes": S, "batch": B, "k": k, "n": n, "field": field, "C": C,
           "erased_natives": sum(1 for r in range(k) if r not in rows)}
    res["enc_batched_us"] = timed(enc_batched, reps)
    res["dec_batched_us"] = timed(dec_batched, reps)
    if B <= 64:
        res["enc_loop_us"] = timed(enc_loop, max(3, reps // 4))
        res["dec_loop_us"] = timed(dec_loop, max(3, reps // 4))
    # both batched launches from one graph replay (launch overhead gone)
    st = torch.cuda.Stream(dev)
    with torch.cuda.stream(st):
        enc_batched()
        dec_batched()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        enc_batched()
        dec_batched()
    res["enc_dec_graph_us"] = timed(g.replay, reps)
    ok = True
    for b in (0, B - 1):
        if field == 16:
            want = gf.field(16).gemm(rs.E, np.ascontiguousarray(data[b].cpu().numpy()).view("<u2"))
            ok = ok and np.array_equal(parity[b].cpu().numpy().view("<u2"), want)
        else:
            want = gf.GF256.gemm(rs.E, data[b].cpu().numpy())
            ok = ok and np.array_equal(parity[b].cpu().numpy(), want)
    ok = ok and torch.equal(out, data)
    res["verified"] = bool(ok)
    obj = B / 1e6
    res["enc_objects_per_s_M"] = round(obj / (res["enc_batched_us"] / 1e6), 3)
    res["dec_objects_per_s_M"] = round(obj / (res["dec_batched_us"] / 1e6), 3)
    res["enc_GBps"] = round(B * k * C / res["enc_batched_us"] / 1e3, 1)
    res["dec_GBps"] = round(B * k * C / res["dec_batched_us"] / 1e3, 1)
    res["enc_dec_graph_GBps"] = round(2 * B * k * C / res["enc_dec_graph_us"] / 1e3, 1)
    for key in list(res):
        if key.endswith("_us"):
            res[key] = round(res[key], 1)
    return res


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--sizes", default="65536,262144,1048576,4194304")
    ap.add_argument("--batches", default="1,16,256")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--code", default="10:14", help="k:n of the code (default the headline's RS(10,14))")
    ap.add_argument("--erase", type=int, default=0, help="natives lost per object (0: the default pattern)")
    ap.add_argument("--field", type=int, default=8, choices=[8, 16], help="16: GF(2^16) symbols (Cauchy code)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    pts = []
    for S in map(int, a.sizes.split(",")):
        for B in map(int, a.batches.split(",")):
            r = point(S, B, a.reps, *(int(v) for v in a.code.split(":")), erase=a.erase, field=a.field)
            print(json.dumps(r), flush=True)
            pts.append(r)
            torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"device": torch.cuda.get_device_name(0), "points": pts}, f, indent=1)
    return 0 if all(r["verified"] for r in pts) else 1


if __name__ == "__main__":
    sys.exit(main())
