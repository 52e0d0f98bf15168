#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs: per case, per kernel, the counter values averaged over
dispatches (plus derived ratios). Usage: scripts/pmc_summary.py gpurun_out/pmc > profiles/.../summary.json"""
import collections
import csv
import glob
import json
import os
import sys


def main(root):
    out = {}
    for f in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
        case = os.path.basename(os.path.dirname(f))
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)", "anon").split("(")[0].replace("void ", "")
            per[name][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[name].add(r["Dispatch_Id"])
        for name, ctr in per.items():
            n = len(disp[name])
            out.setdefault(case, {})[name] = {"dispatches": n, **{k: round(v / n) for k, v in ctr.items()}}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
