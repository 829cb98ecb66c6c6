#!/usr/bin/env python3
"""Folds rocprofv3 --pmc CSVs (one pass per directory) into per-dispatch
counter sums for the kernels whose name contains PATTERN, with per-pop ratios
when POPS is given.  Usage: fold_pmc.py DIR [PATTERN] [POPS=kernel:pops ...]"""
import collections
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "sssp"
    pops = dict(a.split("=", 1)[1].split(":") for a in sys.argv[3:] if a.startswith("POPS="))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for f in sorted(glob.glob(f"{d}/p*/*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if pat not in k:
                continue
            key = (k.split("(")[0].replace("void ", "").split("::")[-1], r["Dispatch_Id"])
            agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
    for (name, disp), v in sorted(agg.items(), key=lambda x: int(x[0][1])):
        print(f"{name} dispatch {disp}")
        for c, x in sorted(v.items()):
            print(f"   {c:28s} {x:.4g}")


if __name__ == "__main__":
    main()
