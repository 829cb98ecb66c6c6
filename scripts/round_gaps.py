#!/usr/bin/env python3
"""Round-boundary gaps from a rocprofv3 --kernel-trace CSV of scripts/round_trace.py:
per round, the GPU idle time from the end of the round's last operation (the fault
word copy) to the start of the next round's first kernel (k_round_init), and the
whole round's span.  Usage: round_gaps.py t_kernel_trace.csv"""
import csv
import re
import statistics as st
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))

    def nm(r):
        m = re.search(r"(k_\w+|__amd_\w+)", r["Kernel_Name"])
        return m.group(1) if m else r["Kernel_Name"][:30]
    gaps, spans = [], []
    inits = [i for i, r in enumerate(rows) if nm(r) == "k_round_init"]
    for a, b in zip(inits, inits[1:]):
        prev = rows[b - 1]
        gaps.append((int(rows[b]["Start_Timestamp"]) - int(prev["End_Timestamp"])) / 1e3)
        spans.append((int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3)
    gaps, spans = gaps[-10:], spans[-10:]
    print(f"rounds {len(gaps)}: boundary gap median {st.median(gaps):.2f} us (min {min(gaps):.2f}, max {max(gaps):.2f}); "
          f"round span median {st.median(spans):.2f} us")


if __name__ == "__main__":
    main()
