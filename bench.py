#!/usr/bin/env python3
"""Headline benchmark: Reed-Solomon encode + decode throughput at k=10, n=14 on 1 GiB per GPU.

Metric (BASELINE.json): "encode+decode throughput (GB/s) at k=10,n=14 on 1 GiB; 1/2/4/8-GPU scaling".

One step on every rank (one process per GPU, torch.distributed/RCCL for N > 1):
  1. encode:  parity[4, C] = E . data[10, C]                          (gfx950 v_perm GF-GEMM)
  2. decode:  4 erasures drawn from a pool of recoverable patterns (natives AND parity erased);
              the decode system is solved ON DEVICE every step (LDS Gauss-Jordan on the e x (e+k)
              systematic system [G[P, erased] | B'], writing the GEMM tables), then the erased
              natives are rebuilt and surviving natives copied in one fused pass into a fresh
              [10, C] output.
C = ceil(2^30 / 10) = 107374183 bytes (odd, as in the reference, src/encode.cu:317). Data is synthetic
random bytes generated in HBM; weights/matrices are the reference Vandermonde. Scaling is weak: every
GPU encodes and decodes its own 1 GiB stripe set (the reference splits one file across GPUs with no
inter-GPU traffic besides a host gather; here E and the erasure-pattern pool are RCCL-broadcast from
rank 0 at setup, and `--gather` adds a per-step parity gather to rank 0 over RCCL).

value = (encoded bytes + decoded bytes) over all ranks / max-over-ranks step time, in GB/s (1e9).
vs_baseline uses the reference's nearest published point (k=8, n=11, 1.1 GB, Tesla C2050:
encode 695.00 ms + decode 1026.68 ms, doc/result-graph/Total-GPU-{en,de}coding-time-3.pdf):
2 * 1,096,310,784 B / 1.72168 s = 1.2736 GB/s. The reference's number includes PCIe copies; the
`--e2e` flag measures the host-pinned end-to-end pipeline as well and adds it to the JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from gpu_rscode_amd import gf  # noqa: E402
from gpu_rscode_amd.models import alloc_rows  # noqa: E402
from gpu_rscode_amd.ops import GemmPlan, decode_system_into_plan, fill_random_  # noqa: E402
from gpu_rscode_amd._native import cpu, hip  # noqa: E402
from gpu_rscode_amd.utils.timing import trace_range  # noqa: E402

BASELINE_GBPS = 2 * 1_096_310_784 / 1.72168 / 1e9  # 1.2736 GB/s


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--bytes", type=int, default=None, help="input bytes per GPU")
    ap.add_argument("--erasures", type=int, default=None)
    ap.add_argument("--vec", type=int, default=None, help="kernel variant: 16-byte groups per lane (ablation)")
    ap.add_argument("--pf", type=int, default=2, help="kernel variant: rows in flight (with --vec)")
    ap.add_argument("--nt", action="store_true", help="kernel variant: non-temporal (with --vec)")
    ap.add_argument("--no-overlap", action="store_true", help="invert on the main stream (no side stream)")
    ap.add_argument("--gather", action="store_true", help="gather parity to rank 0 every step (RCCL)")
    ap.add_argument("--e2e", action="store_true", help="also time the pinned host->device->host pipeline")
    ap.add_argument("--streams", type=int, default=4)
    ap.add_argument("--preset", default="k10n14", choices=sorted(PRESETS),
                    help="BASELINE.json config: k10n14 (headline, #2/#3), k16n20_8g (#4 per GPU), k128n160 (#5), "
                         "k4n6 (the reference's published shape)")
    ap.add_argument("--engine", default="auto", choices=["auto", "valu", "mfma"],
                    help="encode GEMM engine (auto: FP4 matrix cores for wide stripes, v_perm otherwise)")
    ap.add_argument("--graph", action="store_true", help="replay each step from a captured hipGraph")
    a = ap.parse_args()
    pr = PRESETS[a.preset]
    for key, val in pr.items():
        if getattr(a, key) is None:
            setattr(a, key, val)
    return a


# BASELINE.json configs (per-GPU shapes; scaling is weak: every GPU runs one of these)
PRESETS = {
    "k10n14": dict(k=10, n=14, bytes=1 << 30, erasures=4),
    "k16n20_8g": dict(k=16, n=20, bytes=8 << 30, erasures=4),
    "k128n160": dict(k=128, n=160, bytes=1 << 30, erasures=32),
    "k4n6": dict(k=4, n=6, bytes=1_096_310_784, erasures=2),
}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    hip()  # fail loudly if the native extension is missing

    k, n = a.k, a.n
    p = n - k
    C = (a.bytes + k - 1) // k

    # ---- setup: E and the erasure-pattern pool come from rank 0 (RCCL broadcast) -------------
    e_host = gf.GF256.vandermonde_ref(k, p)
    g = gf.GF256.generator(e_host)
    rng = np.random.default_rng(1234)
    pool = []
    while len(pool) < 16:
        erased = sorted(rng.choice(n, size=a.erasures, replace=False).tolist())
        rows = [r for r in range(n) if r not in erased]
        if any(e < k for e in erased) and cpu().decode_matrix(g.tobytes(), k, rows) is not None:
            pool.append(rows)
    e_dev = torch.from_numpy(e_host.copy()).to(dev)
    g_dev = torch.from_numpy(np.ascontiguousarray(g)).to(dev)
    pool_dev = torch.tensor(pool, dtype=torch.int32, device=dev)
    if world > 1:
        dist.broadcast(e_dev, 0)
        dist.broadcast(g_dev, 0)
        dist.broadcast(pool_dev, 0)
    pool = pool_dev.cpu().tolist()
    e_mat = e_dev.cpu().numpy()

    data = alloc_rows(k, C, dev)
    fill_random_(data.as_strided((data.untyped_storage().nbytes(),), (1,)), seed=rank + 1)
    parity = alloc_rows(p, C, dev)
    out = alloc_rows(k, C, dev)

    enc = GemmPlan(data, parity, e_mat, engine=a.engine)
    stripe = [data[i] for i in range(k)] + [parity[i] for i in range(p)]
    dec = []
    for rows in pool:
        erased = [i for i in range(k) if i not in rows]
        ins = [stripe[r] for r in rows]
        copies = [out[r] if r < k else None for r in rows]
        plan = GemmPlan(ins, [out[i] for i in erased], copies=copies, device_tables=True)
        plan.rows_dev = torch.tensor(rows, dtype=torch.int32, device=dev)
        plan.erased_dev = torch.tensor(erased, dtype=torch.int32, device=dev)
        plan.status = torch.zeros(1, dtype=torch.int32, device=dev)
        dec.append(plan)
    gathered = None
    if a.graph and a.gather:
        raise SystemExit("--graph and --gather are exclusive")
    if a.gather and world > 1 and rank == 0:
        gathered = [torch.empty_like(parity.as_strided((p * parity.stride(0),), (1,))) for _ in range(world)]

    stream = torch.cuda.Stream(dev)  # a non-default stream (hipGraph capture needs one)
    torch.cuda.set_stream(stream)
    side = torch.cuda.Stream(dev)  # decode-system inversion overlaps the encode GEMM
    inv_done = torch.cuda.Event()
    kv = dict(vec=a.vec, pf=a.pf, nt=a.nt)

    def step(i: int):
        plan = dec[i % len(dec)]
        inv_stream = stream if a.no_overlap else side
        if not a.no_overlap:
            side.wait_stream(stream)  # the previous step's decode has consumed this plan's tables
        # the decode system solved on device (e x (e+k) Gauss-Jordan on [G[P, erased] | B'])
        # writing the decode tables (and, on the matrix-core engine, the bit-matrix) into the plan
        decode_system_into_plan(g_dev, plan.rows_dev, plan.erased_dev, plan, status=plan.status, stream=inv_stream)
        if not a.no_overlap:
            inv_done.record(side)
        enc.run(**kv)
        if not a.no_overlap:
            stream.wait_event(inv_done)
        plan.run(**kv)
        if a.gather and world > 1:
            flat = parity.as_strided((p * parity.stride(0),), (1,))
            dist.gather(flat, gathered if rank == 0 else None, dst=0)

    with trace_range("bench/warmup"):
        for i in range(max(a.warmup, len(dec) if a.graph else 0)):
            step(i)
        torch.cuda.synchronize()
    if a.graph:
        # one captured graph per decode pattern: encode GEMM, side-stream inversion, decode GEMM
        graphs = []
        for i in range(len(dec)):
            gph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gph, stream=stream):
                step(i)
            graphs.append(gph)
        torch.cuda.synchronize()
        run_step = lambda i: graphs[i % len(graphs)].replay()  # noqa: E731
    else:
        run_step = step
    timed = trace_range("bench/timed")  # roctx range opened before the bracket, closed after it
    timed.__enter__()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        run_step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    timed.__exit__(None, None, None)
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    # ---- verification (outside the timed region) ----------------------------------------------
    last = dec[(a.steps - 1) % len(dec)]
    ok = int(last.status.item()) == 0 and torch.equal(out, data)
    cols = min(C, 1 << 16)
    want = gf.GF256.gemm(e_mat, data[:, :cols].cpu().numpy())
    ok = ok and np.array_equal(parity[:, :cols].cpu().numpy(), want)
    okt = torch.tensor([1 if ok else 0], device=dev)
    if world > 1:
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    ok = bool(okt.item())

    ms = elapsed / a.steps * 1e3
    bytes_per_step = 2 * k * C * world  # encoded input + decoded output, all ranks
    gbps = bytes_per_step / (ms / 1e3) / 1e9
    metric = "encode+decode throughput (GB/s) at k=10,n=14 on 1 GiB; 1/2/4/8-GPU scaling"
    if a.preset != "k10n14":
        metric = f"encode+decode throughput (GB/s) at k={k},n={n} on {a.bytes / 2**30:.3g} GiB per GPU"
    rec = {
        "metric": metric,
        "value": round(gbps, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(gbps / BASELINE_GBPS, 1),
        "dtype": "uint8 (GF(2^8) symbols)",
        "data": "synthetic (device-generated random bytes)",
        "config": {"model": f"RS(k={k},n={n}) reference Vandermonde, GF(2^8) poly 0x11D",
                   "global_batch": f"{a.bytes} B per GPU ({k} x {C} B chunks)", "seq_len": C,
                   "parallelism": f"dp{world} (stripe-sharded, RCCL broadcast of E)",
                   "erasures": a.erasures, "decode_invert": "device Gauss-Jordan (systematic e x (e+k) system) per step",
                   "gather": bool(a.gather), "engine": enc.engine, "graph": bool(a.graph), "preset": a.preset},
        "verified": ok,
        "baseline": {"gbps": round(BASELINE_GBPS, 4), "source": "k=8,n=11 1.1 GB Tesla C2050 (nearest published)"},
    }
    if a.e2e and rank == 0:
        rec["e2e"] = e2e(a, k, p, C, e_mat, dev)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


def e2e(a, k, p, C, e_mat, dev):
    """Reference-comparable timing: pinned host rows -> H2D -> kernel -> D2H, -s streams."""
    host = torch.empty(k * C, dtype=torch.uint8, pin_memory=True)
    host.copy_(torch.randint(0, 256, (k * C,), dtype=torch.uint8))
    par = torch.empty(p * C, dtype=torch.uint8, pin_memory=True)
    ins = [host.data_ptr() + j * C for j in range(k)]
    outs = [par.data_ptr() + i * C for i in range(p)]
    res = hip().gemm_host([dev.index], ins, outs, np.ascontiguousarray(e_mat).tobytes(), C, a.streams, 32 << 20, 0,
                          False)
    res = hip().gemm_host([dev.index], ins, outs, np.ascontiguousarray(e_mat).tobytes(), C, a.streams, 32 << 20, 0,
                          False)
    d = res["devices"][0]
    return {"encode_ms_total": round(d["ms_total"], 3), "encode_ms_stream": round(d["ms_stream"], 3),
            "encode_MBps_total": round(k * C / 1048576 / (d["ms_total"] / 1e3), 1),
            "streams": a.streams}


if __name__ == "__main__":
    main()
