#!/usr/bin/env python3
"""Where a timed loop's fixed cost goes: the kernels at the start and the end of a bench timed
region, from one rocprofv3 run with --kernel-trace --marker-trace (csv).

  rocprofv3 --kernel-trace --marker-trace --output-format csv -d DIR -o run -- python3 bench.py ...
  python scripts/loop_edges.py DIR [--label bench/] [--edge 10] [--json out.json]

The timed region is the roctx range bench.py opens around each timed loop (trace_range
"bench/<mode>"); the first such range is the headline. Reports the host range, the first kernel's
start and the last kernel's end relative to it, the GPU-idle time inside the range (no kernel
running), and the first and last `--edge` kernels with their start offsets, durations and the idle
gap before each.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re


def _rows(d: str, suffix: str) -> list[dict]:
    files = glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True)
    out = []
    for f in files:
        with open(f, newline="") as fh:
            out += list(csv.DictReader(fh))
    return out


def short(name: str) -> str:
    """kernel name + template arguments, without namespaces and parameters"""
    n = name.replace("(anonymous namespace)::", "")
    m = re.search(r"([A-Za-z_][A-Za-z0-9_]*)(<[^()]*>)?\(", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:70]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--label", default="bench/")
    ap.add_argument("--edge", type=int, default=10)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    kern = sorted(({"name": r["Kernel_Name"], "start": int(r["Start_Timestamp"]), "end": int(r["End_Timestamp"])}
                   for r in _rows(a.dir, "kernel_trace.csv")), key=lambda r: r["start"])
    marks = [r for r in _rows(a.dir, "marker_api_trace.csv") if r.get("Function", "").startswith(a.label)]
    if not marks:
        raise SystemExit(f"no marker range starting with {a.label!r}")
    marks.sort(key=lambda r: int(r["Start_Timestamp"]))
    m = marks[0]
    t0, t1 = int(m["Start_Timestamp"]), int(m["End_Timestamp"])
    inside = [k for k in kern if k["end"] > t0 and k["start"] < t1]
    # GPU-idle time inside the range (union of kernel intervals)
    busy, cur_s, cur_e = 0, None, None
    for k in inside:
        s, e = max(k["start"], t0), min(k["end"], t1)
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s

    def listing(ks):
        out, prev_end = [], None
        for k in ks:
            gap = None if prev_end is None else (k["start"] - prev_end) / 1e3
            out.append({"kernel": short(k["name"]), "start_us": round((k["start"] - t0) / 1e3, 1),
                        "dur_us": round((k["end"] - k["start"]) / 1e3, 1),
                        "idle_before_us": None if gap is None else round(max(gap, 0.0), 1)})
            prev_end = k["end"] if prev_end is None else max(prev_end, k["end"])
        return out

    rep = {
        "range": m["Function"], "host_ms": round((t1 - t0) / 1e6, 4), "kernels": len(inside),
        "first_kernel_start_us": round((inside[0]["start"] - t0) / 1e3, 1) if inside else None,
        "last_kernel_end_to_range_end_us": round((t1 - max(k["end"] for k in inside)) / 1e3, 1) if inside else None,
        "gpu_idle_in_range_us": round((t1 - t0 - busy) / 1e3, 1),
        "first": listing(inside[:a.edge]), "last": listing(inside[-a.edge:]),
    }
    print(json.dumps(rep, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
