#!/usr/bin/env python3
"""Times shd_topology_latency_rows_frontier (the bucketed frontier SSSP) on
the C2 graph (V = 20k, H = 50k) and, with --c4, all rows of C4 (V = 100k,
H = 200k; 60 GB of latencies).  Usage: frontier_probe.py [--c4]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from shadow_amd import Topology, scenario, synth
    cfgs = [("C2", 20_000, 50_000, 0x5EED0002)] + ([("C4", 100_000, 200_000, 0x5EED0004)] if "--c4" in sys.argv else [])
    for name, V, H, seed in cfgs:
        top = Topology(synth.sparse_graph_gml(V, seed))
        scenario.register_hosts(top, H, seed=1)
        A = top.slot_count()
        d = torch.empty(A * A, dtype=torch.float64, device="cuda")
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            top.latency_rows_frontier(0, A, d.data_ptr())
            torch.cuda.synchronize()
            print(f"{name} frontier latencies, {A} rows x {A}: {time.perf_counter() - t0:.3f}s", flush=True)
        del d
        top.close()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
