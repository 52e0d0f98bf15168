#!/usr/bin/env python3
"""Timeline of a rocprofv3 kernel trace: which streams the RCCL kernels ran on and how much of their
time overlapped the GF-GEMM kernels.

  rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python3 bench.py --force-pg ...
  python scripts/trace_overlap.py DIR [--last 40] [--out timeline.txt]

Prints, for RCCL kernels (name contains "nccl"): count, total time, the streams/queues they used,
and the fraction of their busy time during which a gfrs GEMM kernel (gf_gemm*) was also running on
another stream — the evidence that collectives overlap compute. Then the last N kernels as a
timeline (start/end relative to the first of them, queue, stream, short name).
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import re
import sys


def load(path: str) -> list[dict]:
    files = [path] if os.path.isfile(path) else glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no *kernel_trace.csv under {path}")
    rows = []
    for f in files:
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                rows.append(dict(name=r["Kernel_Name"], start=int(r["Start_Timestamp"]), end=int(r["End_Timestamp"]),
                                 queue=r.get("Queue_Id", "?"), stream=r.get("Stream_Id", "?")))
    rows.sort(key=lambda r: r["start"])
    return rows


def short(name: str) -> str:
    name = name.replace("gfrs::(anonymous namespace)::", "gfrs::anon::")
    return re.sub(r"\(.*\)$", "", name)[:90]


def is_rccl(name: str) -> bool:
    return "nccl" in name.lower()


def is_gemm(name: str) -> bool:
    return "gf_gemm" in name


def union_overlap(a0: int, a1: int, spans: list[tuple[int, int]]) -> int:
    """Length of [a0, a1) covered by the union of spans (sorted by start)."""
    cov, cur0, cur1 = 0, None, None
    for s0, s1 in spans:
        s0, s1 = max(s0, a0), min(s1, a1)
        if s1 <= s0:
            continue
        if cur1 is None or s0 > cur1:
            if cur1 is not None:
                cov += cur1 - cur0
            cur0, cur1 = s0, s1
        else:
            cur1 = max(cur1, s1)
    if cur1 is not None:
        cov += cur1 - cur0
    return cov


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("trace", help="rocprofv3 output directory or a kernel_trace.csv")
    ap.add_argument("--last", type=int, default=40)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    rows = load(a.trace)
    rccl = [r for r in rows if is_rccl(r["name"])]
    gemm = [r for r in rows if is_gemm(r["name"])]
    lines = []
    busy = sum(r["end"] - r["start"] for r in rccl)
    lines.append(f"kernels: {len(rows)}  gemm: {len(gemm)}  rccl: {len(rccl)}")
    if rccl:
        streams = sorted({(r["queue"], r["stream"]) for r in rccl})
        gstreams = sorted({(r["queue"], r["stream"]) for r in gemm})
        ov = 0
        for r in rccl:
            others = [(g["start"], g["end"]) for g in gemm if (g["queue"], g["stream"]) != (r["queue"], r["stream"])]
            ov += union_overlap(r["start"], r["end"], others)
        names = sorted({short(r["name"]) for r in rccl})
        lines.append(f"rccl kernels: {', '.join(names)}")
        lines.append(f"rccl (queue, stream): {streams}; gemm (queue, stream): {gstreams}")
        lines.append(f"rccl busy: {busy / 1e3:.1f} us total, {busy / max(1, len(rccl)) / 1e3:.1f} us mean; "
                     f"overlapped by a GEMM on another stream: {ov / 1e3:.1f} us ({100.0 * ov / max(1, busy):.1f} %)")
    tail = rows[-a.last:]
    if tail:
        t0 = tail[0]["start"]
        lines.append(f"\nstart_us   end_us   dur_us  queue stream kernel   (last {len(tail)} kernels)")
        for r in tail:
            lines.append(f"{(r['start'] - t0) / 1e3:8.1f} {(r['end'] - t0) / 1e3:8.1f} {(r['end'] - r['start']) / 1e3:8.1f}"
                         f"  q{r['queue']:<4} s{r['stream']:<5} {short(r['name'])}")
    text = "\n".join(lines)
    print(text)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(text + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
