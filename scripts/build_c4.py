#!/usr/bin/env python3
"""Builds a routing table once, as bench.py's legs do -- a target for PMC
passes over one slab-kernel launch (scripts/pmc_r03.sh).  Default: C4 (V=100k,
H=200k, all 86,603 rows); `build_c4.py V H SEED` for another sparse config
(C2: 20000 50000 0x5EED0002), `build_c4.py complete V H SEED` for a complete
graph (C1: complete 1000 5000 0x5EED0001; rebuilt 5 times, as the bench)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from shadow_amd import Topology, scenario, synth
    import torch
    args = sys.argv[1:]
    complete = bool(args) and args[0] == "complete"
    if complete:
        args = args[1:]
    V, H, seed = (int(args[0]), int(args[1]), int(args[2], 0)) if len(args) > 2 else (100_000, 200_000, 0x5EED0004)
    top = Topology(synth.complete_graph_gml(V, seed) if complete else synth.sparse_graph_gml(V, seed))
    scenario.register_hosts(top, H, seed=1)
    A = top.slot_count()
    tab = top.alloc_table(A * A * 16)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5 if complete else 1):
        top.build_rows_device(0, A, tab.ptr)
    torch.cuda.synchronize()
    print(f"build V={V} H={H} A={A}: {time.perf_counter() - t0:.2f}s", flush=True)


if __name__ == "__main__":
    main()
