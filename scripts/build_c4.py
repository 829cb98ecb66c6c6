#!/usr/bin/env python3
"""Builds the C4 routing table once (V=100k, H=200k, all 86,603 rows into a
device table), as bench.py's C4 leg does -- a target for PMC passes over the
C4 slab-kernel launch (scripts/r02_final_pmc.sh)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from shadow_amd import Topology, scenario, synth
    import torch
    top = Topology(synth.sparse_graph_gml(100_000, 0x5EED0004))
    scenario.register_hosts(top, 200_000, seed=1)
    A = top.slot_count()
    tab = top.alloc_table(A * A * 16)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    top.build_rows_device(0, A, tab.ptr)
    torch.cuda.synchronize()
    print(f"C4 build A={A}: {time.perf_counter() - t0:.2f}s", flush=True)


if __name__ == "__main__":
    main()
