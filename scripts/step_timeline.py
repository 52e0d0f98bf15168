#!/usr/bin/env python3
"""Where a bench step's time goes, from a rocprofv3 kernel trace (any preset).

  rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 bench.py --no-e2e ...
  python scripts/step_timeline.py DIR [--gemm gf_gemm] [--skip-ms 50] [--json out.json]

The GEMM kernels (names matching --gemm) are merged into busy intervals over the traced window
(after --skip-ms of warm-up; lanes that overlap count once). Reported: the window, the fraction of
it the GEMMs keep the GPU busy, the idle gaps between busy intervals (count, median, p90, max, sum),
per kernel name the count and median / max duration, and for every other kernel (plan build,
solve, broadcast, fills) the same plus how much of its time overlapped a GEMM. The idle sum is what
a perfect schedule could still win back; the rest of the step is the kernels themselves.
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


def short(name: str) -> str:
    name = re.sub(r"^(void )?", "", name).replace("(anonymous namespace)::", "").replace("gfrs::", "")
    return name.split("(", 1)[0][:120]  # drop the argument list


def merge(iv: list[tuple[int, int]]) -> list[list[int]]:
    out: list[list[int]] = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def overlap(a: int, b: int, busy: list[list[int]]) -> int:
    return sum(max(0, min(b, y) - max(a, x)) for x, y in busy)


def stats(xs: list[float]) -> dict | None:
    if not xs:
        return None
    s = sorted(xs)
    return {"n": len(s), "median": round(statistics.median(s), 2), "p90": round(s[int(0.9 * (len(s) - 1))], 2),
            "max": round(s[-1], 2), "sum": round(sum(s), 1)}


def analyse(rows: list[dict], gemm_re: str, skip_ms: float) -> dict:
    rx = re.compile(gemm_re)
    gem = [r for r in rows if rx.search(r["name"])]
    if not gem:
        raise SystemExit(f"no kernel matches {gemm_re!r}")
    t0 = gem[0]["start"] + int(skip_ms * 1e6)
    gem = [r for r in gem if r["start"] >= t0]
    t1 = max(r["end"] for r in gem)
    busy = merge([(r["start"], r["end"]) for r in gem])
    window = t1 - busy[0][0]
    gaps = [(busy[i + 1][0] - busy[i][1]) / 1e3 for i in range(len(busy) - 1)]
    per: dict[str, list[float]] = {}
    for r in gem:
        per.setdefault(short(r["name"]), []).append((r["end"] - r["start"]) / 1e3)
    others: dict[str, dict] = {}
    for r in rows:
        if rx.search(r["name"]) or r["start"] < busy[0][0] or r["start"] > t1:
            continue
        o = others.setdefault(short(r["name"]), {"us": [], "overlap": 0, "total": 0})
        o["us"].append((r["end"] - r["start"]) / 1e3)
        o["overlap"] += overlap(r["start"], r["end"], busy)
        o["total"] += r["end"] - r["start"]
    return {
        "window_ms": round(window / 1e6, 3),
        "gemm_busy_fraction": round(sum(b - a for a, b in busy) / window, 4),
        "gaps_us": stats(gaps),
        "gemm_kernels": {k: stats(v) for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))},
        "other_kernels": {k: {**stats(v["us"]), "overlapped_fraction": round(v["overlap"] / max(1, v["total"]), 3)}
                          for k, v in sorted(others.items(), key=lambda kv: -sum(kv[1]["us"]))},
    }


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("trace")
    ap.add_argument("--gemm", default=r"gf_gemm", help="regex of the GEMM kernel names")
    ap.add_argument("--skip-ms", type=float, default=50.0, help="leading trace time to ignore (warm-up)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    res = analyse(load(a.trace), a.gemm, a.skip_ms)
    print(json.dumps(res, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
