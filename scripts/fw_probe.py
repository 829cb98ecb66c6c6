#!/usr/bin/env python3
"""Times shd_topology_latency_table_fw (blocked min-plus Floyd-Warshall) on
the C1 graph; run under rocprofv3 --kernel-trace --stats for per-kernel times."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from shadow_amd import Topology, scenario, synth
    V = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    top = Topology(synth.complete_graph_gml(V, 0x5EED0001))
    scenario.register_hosts(top, 5 * V, seed=1)
    A = top.slot_count()
    d = torch.empty(A * A, dtype=torch.float64, device="cuda")
    top.latency_table_fw(d.data_ptr())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        top.latency_table_fw(d.data_ptr())
    torch.cuda.synchronize()
    print(f"min-plus latencies V={V} A={A}: {(time.perf_counter() - t0) / 5 * 1e3:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
