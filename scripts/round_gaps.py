#!/usr/bin/env python3
"""Round-boundary gaps from a rocprofv3 --kernel-trace CSV of scripts/round_trace.py:
per round, the GPU idle time from the end of the previous round's last operation
(the fault word's store or copy) to the start of the round's first kernel
(k_round_init, or the scatter itself when the round's resets were left done by the
round before), and the span from one round's scatter to the next.
Usage: round_gaps.py t_kernel_trace.csv"""
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
    big = max(int(r["Grid_Size_X"]) for r in rows if nm(r) == "k_part_scatter")
    sc = [i for i, r in enumerate(rows) if nm(r) == "k_part_scatter" and int(r["Grid_Size_X"]) == big]
    gaps, spans = [], []
    for a, b in zip(sc, sc[1:]):
        first = b - 1 if nm(rows[b - 1]) == "k_round_init" else b
        gaps.append((int(rows[first]["Start_Timestamp"]) - int(rows[first - 1]["End_Timestamp"])) / 1e3)
        spans.append((int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3)
    gaps, spans = gaps[-10:], spans[-10:]
    print(f"rounds {len(gaps)}: boundary gap median {st.median(gaps):.2f} us (min {min(gaps):.2f}, max {max(gaps):.2f}); "
          f"round span (scatter to scatter) median {st.median(spans):.2f} us")


if __name__ == "__main__":
    main()
