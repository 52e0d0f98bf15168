#!/usr/bin/env python3
"""Summarise rocprofv3 SQLite outputs (``run_results.db``, the default format of this rocprofv3):
per kernel (name filter) the dispatch count, median / total duration and, for PMC runs, the
counters averaged per dispatch plus derived clock, MFMA-pipe utilisation and VALU per MFMA (as
scripts/pmc_clock.py does for CSV outputs).

    python scripts/rocpd_summary.py FILTER DB [DB ...]
"""
from __future__ import annotations

import collections
import json
import sqlite3
import sys


def summarise(path: str, filt: str) -> dict:
    db = sqlite3.connect(path)
    durs = collections.defaultdict(list)
    for name, dur in db.execute("select name, duration from kernels"):
        if filt in name:
            durs[name].append(dur / 1e3)
    ctr = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    try:
        rows = db.execute("select kernel_name, dispatch_id, counter_name, value from counters_collection").fetchall()
    except sqlite3.DatabaseError:
        rows = []
    for name, d, cname, val in rows:
        if filt in name:
            ctr[name][cname] += float(val)
            disp[name].add(d)
    out = {}
    for name in sorted(set(durs) | set(ctr)):
        ts = sorted(durs.get(name, []))
        r = {"dispatches": len(ts), "median_us": round(ts[len(ts) // 2], 1) if ts else None,
             "total_us": round(sum(ts), 1)}
        n = max(1, len(disp.get(name, ())))
        c = {k: v / n for k, v in ctr.get(name, {}).items()}
        if c:
            cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8
            if cyc and r["median_us"]:
                r["clock_GHz"] = round(cyc / r["median_us"] / 1e3, 3)
                if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                    r["mfma_pipe_util"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc), 3)
            if c.get("SQ_INSTS_MFMA"):
                r["valu_per_mfma"] = round(c.get("SQ_INSTS_VALU", 0) / c["SQ_INSTS_MFMA"], 2)
            r["counters"] = {k: round(v) for k, v in c.items()}
        out[name[:160]] = r
    return out


if __name__ == "__main__":
    filt = sys.argv[1]
    print(json.dumps({p: summarise(p, filt) for p in sys.argv[2:]}, indent=1))
