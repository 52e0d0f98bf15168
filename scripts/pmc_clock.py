#!/usr/bin/env python3
"""Per rocprofv3 output directory (kernel trace + one PMC pass): median wall time, effective clock
(GRBM_GUI_ACTIVE / 8 XCDs / wall), MFMA-pipe utilisation and VALU per MFMA of the kernels whose
name contains a filter string. Usage: scripts/pmc_clock.py FILTER DIR..."""
import collections
import csv
import glob
import json
import sys


def summarise(d, filt):
    ctr, disp = collections.defaultdict(float), set()
    for f in glob.glob(d + "/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if filt in r["Kernel_Name"]:
                ctr[r["Counter_Name"]] += float(r["Counter_Value"])
                disp.add(r["Dispatch_Id"])
    ts = []
    for f in glob.glob(d + "/**/run_kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if filt in r["Kernel_Name"]:
                ts.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    n = max(1, len(disp))
    c = {k: v / n for k, v in ctr.items()}
    t = sorted(ts)[len(ts) // 2] if ts else 0.0
    cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8
    waves = c.get("SQ_WAVES")
    res = {"dir": d, "dispatches": len(disp), "median_us": round(t, 1)}
    if t and cyc:
        res["clock_GHz"] = round(cyc / t / 1e3, 3)
        res["kernel_cycles"] = round(cyc)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            res["mfma_pipe_util"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc), 3)
    if c.get("SQ_INSTS_MFMA"):
        res["valu_per_mfma"] = round(c.get("SQ_INSTS_VALU", 0) / c["SQ_INSTS_MFMA"], 2)
        res["mfma_per_dispatch"] = round(c["SQ_INSTS_MFMA"])
    res["counters"] = {k: round(v) for k, v in c.items()}
    return res


if __name__ == "__main__":
    filt = sys.argv[1]
    print(json.dumps([summarise(d, filt) for d in sys.argv[2:]], indent=1))
