#!/usr/bin/env python3
"""Folds a scripts/ubench_mixed log into profiles/r03_request_ceiling.json:
one key per case, "<footprint MB>MB_<write %>pct_writes" -> G requests/s.
Usage: scripts/ceiling.py LOG OUT.json"""
import json
import re
import sys


def main():
    log, out = sys.argv[1], sys.argv[2]
    res = {}
    for ln in open(log):
        m = re.match(r"footprint\s+(\d+) MB\s+writes\s+([\d.]+) %\s+([\d.]+) ms\s+([\d.]+) G requests/s", ln.strip())
        if m:
            res[f"{int(m.group(1))}MB_{float(m.group(2)):g}pct_writes"] = float(m.group(4))
    res["_source"] = f"scripts/ubench_mixed.hip on the GPU box ({log.split('/')[-1]}): independent random 16-B " \
                     "requests, median of 7 launches"
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
