#!/usr/bin/env python3
"""Summarise a tools/profile.sh output directory: per kernel, average duration (kernel trace)
and the average of every PMC counter per dispatch; HBM bytes per dispatch are
FETCH_SIZE*2 (gfx950 reports half of a wide streaming read, MI355X_MICROARCH.md §HBM) +
WRITE_SIZE, both in KiB units.  Usage: tools/prof_summary.py gpurun_out/prof_<tag> [--json out]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(r8::Args)")[0].split("(")[0] if "k_pass<" not in name else name.split("(")[0]


def main():
    d = sys.argv[1]
    kt = defaultdict(list)
    for f in glob.glob(os.path.join(d, "kt", "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            kt[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    pmc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "pmc_*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k in sorted(set(kt) | set(pmc)):
        ent = {}
        if kt.get(k):
            ent["calls"] = len(kt[k])
            ent["avg_ms"] = sum(kt[k]) / len(kt[k])
        for c, v in pmc.get(k, {}).items():
            ent[c] = sum(v) / len(v)
        if "FETCH_SIZE" in ent and "WRITE_SIZE" in ent:
            ent["hbm_bytes_corrected"] = (2 * ent["FETCH_SIZE"] + ent["WRITE_SIZE"]) * 1024
        out[k] = ent
    for k, ent in out.items():
        print(k)
        for c, v in sorted(ent.items()):
            print(f"    {c:28s} {v:,.4f}")
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
