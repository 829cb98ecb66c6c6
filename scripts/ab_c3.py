#!/usr/bin/env python3
"""Prints ms/round and per-stage times from bench.py JSON lines in the given
logs (A/B runs of C3-only benches).  Usage: ab_c3.py LOG..."""
import json
import sys

for f in sys.argv[1:]:
    try:
        line = [x for x in open(f) if x.startswith("{")][0]
    except (OSError, IndexError):
        print(f, "no bench line")
        continue
    d = json.loads(line)
    st = {k: round(v, 4) for k, v in d["roofline"]["per_stage_ms"].items()}
    print(f, round(d["ms_per_step"], 4), st)
