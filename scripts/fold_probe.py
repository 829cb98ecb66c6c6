#!/usr/bin/env python3
"""In-process A/B of a path-counter fold knob: per block, K C3 rounds log
their kept packets' owner pairs (untimed), then shd_topology_path_counts_sync
folds the K logs into the counters (timed, wall).  At the end every pair's
count must be the number of rounds times one round's.
Usage: fold_probe.py ENV V1 V2 ... (K = FOLD_K, default 20)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from shadow_amd import Topology, scenario, synth
    H, V, P = 100_000, 20_000, 10_000_000
    K = int(os.environ.get("FOLD_K", "20"))
    dev = torch.device("cuda", 0)
    top = Topology(synth.sparse_graph_gml(V, 0x5EED0002))
    _, states, _ = scenario.register_hosts(top, H, seed=1)
    A = top.slot_count()
    table = top.alloc_table(A * A * 16)
    top.build_rows_device(0, A, table.ptr)
    top.adopt_table_device(table.ptr)
    top.touch_all()
    pk = synth.packet_batch(P, H, 0x5EED0003, 100_000_000, 10_000_000, states)
    d_recs = torch.from_numpy(pk.view(np.uint8)).to(dev)
    d_out = torch.empty(P * 32, dtype=torch.uint8, device=dev)
    d_off = torch.empty(H + 1, dtype=torch.int32, device=dev)
    d_status = torch.empty(P, dtype=torch.uint8, device=dev)
    d_cnt = torch.empty(2, dtype=torch.int64, device=dev)
    name, vals = sys.argv[1], sys.argv[2:]
    top.process_device(d_recs.data_ptr(), P, 110_000_000, 10**15, 0, d_out.data_ptr(), d_off.data_ptr(),
                       d_status.data_ptr(), d_cnt.data_ptr(), 0)
    top.path_counts_sync()
    one = top.path_packet_counts()  # one round's counts (every round counts the same)
    for rep in range(3):
        for v in vals:
            if v == "-":
                os.environ.pop(name, None)
            else:
                os.environ[name] = v
            for _ in range(K):
                top.process_device(d_recs.data_ptr(), P, 110_000_000, 10**15, 0, d_out.data_ptr(), d_off.data_ptr(),
                                   d_status.data_ptr(), d_cnt.data_ptr(), 0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            top.path_counts_sync()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) * 1e3
            print(f"{name}={v} rep {rep}: fold of {K} rounds {dt:.3f} ms ({dt / K:.4f} ms per round)", flush=True)
    c = top.path_packet_counts()
    rounds = 1 + 3 * len(vals) * K
    print(f"counts after {rounds} rounds == {rounds} x one round's, every pair: "
          f"{bool(np.array_equal(c, one * np.uint64(rounds)))}", flush=True)


if __name__ == "__main__":
    main()
