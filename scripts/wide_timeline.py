#!/usr/bin/env python3
"""Per-step timeline of a wide-stripe bench run from a rocprofv3 kernel trace.

  rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 bench.py --preset k128n160 --lanes 1 ...
  python scripts/wide_timeline.py DIR [--json out.json]

Classifies the kernels of the timed steps — encode GEMM (FP4 kernels without fused copies),
decode GEMM (fused-copy FP4 kernel, template COPY = true), decode-system solve
(gf_decode_system_kernel) — and reports, per decode: the solve that built its plan (the last one
that ended before the decode started), whether it ended before the decode began, how long the GPU
waited between the previous GEMM's end and the decode's start, and each kernel's own duration.
Summary: median / max of each, the fraction of decodes whose solve was off the critical path, and
the GEMM busy fraction of the traced window (sum of GEMM durations / wall, lanes overlapping count
once).
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
import statistics


def load(path: str) -> list[dict]:
    files = [path] if os.path.isfile(path) else glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no *kernel_trace.csv under {path}")
    rows = []
    for f in files:
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                rows.append(dict(name=r["Kernel_Name"], start=int(r["Start_Timestamp"]), end=int(r["End_Timestamp"])))
    rows.sort(key=lambda r: r["start"])
    return rows


def kind(name: str) -> str | None:
    if "gf_decode_system_kernel" in name:
        return "solve"
    m = re.search(r"gf_gemm_fp4(ar|tm)?_kernel<([^>]*)>", name)
    if not m:
        return None
    args = [a.strip() for a in m.group(2).split(",")]
    # fp4ar<MGW, WPG, UNI, COPY, R, ...>; fp4<MG, UNI, COPY, R, KS>; fp4tm<MG, UNI, COPY>
    copy = args[3] if m.group(1) == "ar" else args[2]
    return "decode" if copy == "true" else "encode"


def analyse(rows: list[dict], skip: int) -> dict:
    ks = [dict(r, kind=kind(r["name"])) for r in rows]
    ks = [r for r in ks if r["kind"]]
    decodes = [r for r in ks if r["kind"] == "decode"][skip:]
    solves = [r for r in ks if r["kind"] == "solve"]
    gemms = [r for r in ks if r["kind"] in ("encode", "decode")]
    per = []
    for d in decodes:
        before = [s for s in solves if s["start"] < d["start"]]
        s = before[-1] if before else None
        prev_end = max((g["end"] for g in gemms if g["end"] <= d["start"] and g is not d), default=d["start"])
        per.append({"decode_us": (d["end"] - d["start"]) / 1e3,
                    "solve_us": (s["end"] - s["start"]) / 1e3 if s else None,
                    "solve_done_before_decode": bool(s and s["end"] <= d["start"]),
                    "solve_end_to_decode_start_us": (d["start"] - s["end"]) / 1e3 if s else None,
                    "gap_before_decode_us": max(0.0, (d["start"] - prev_end) / 1e3)})
    enc = [(r["end"] - r["start"]) / 1e3 for r in ks if r["kind"] == "encode"][skip:]
    if decodes:
        t0, t1 = decodes[0]["start"], decodes[-1]["end"]
        busy, cur = 0, None
        for g in sorted((g for g in gemms if g["end"] > t0 and g["start"] < t1), key=lambda g: g["start"]):
            a, b = max(g["start"], t0), min(g["end"], t1)
            if cur is None or a > cur[1]:
                if cur:
                    busy += cur[1] - cur[0]
                cur = [a, b]
            else:
                cur[1] = max(cur[1], b)
        if cur:
            busy += cur[1] - cur[0]
        window = t1 - t0
    else:
        busy = window = 0

    def stats(xs):
        xs = [x for x in xs if x is not None]
        return {"median": round(statistics.median(xs), 1), "max": round(max(xs), 1), "n": len(xs)} if xs else None

    return {
        "decodes": len(per),
        "encode_us": stats(enc),
        "decode_us": stats([p["decode_us"] for p in per]),
        "solve_us": stats([p["solve_us"] for p in per]),
        "solve_off_critical_path": sum(p["solve_done_before_decode"] for p in per) / max(1, len(per)),
        "gap_before_decode_us": stats([p["gap_before_decode_us"] for p in per]),
        "gemm_busy_fraction": round(busy / window, 4) if window else None,
        "per_decode": per,
    }


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=4, help="leading decodes to ignore (warmup)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    res = analyse(load(a.trace), a.skip)
    summary = {k: v for k, v in res.items() if k != "per_decode"}
    print(json.dumps(summary, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
