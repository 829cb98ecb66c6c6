#!/usr/bin/env python3
"""Launch-overhead probe for the C3 round (dev tool): the same 10M-packet
round launched eagerly (shd_round_process_device per round) and replayed from
a HIP graph captured around one call; prints ms per round for both and checks
the outputs are identical."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from shadow_amd import Topology, scenario, synth
    H, V, P = 100_000, 20_000, 10_000_000
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
    stream = torch.cuda.Stream(dev)

    def rnd(s):
        top.process_device(d_recs.data_ptr(), P, 110_000_000, 10**15, 0, d_out.data_ptr(), d_off.data_ptr(),
                           d_status.data_ptr(), d_cnt.data_ptr(), s.cuda_stream)

    with torch.cuda.stream(stream):
        for _ in range(3):
            rnd(stream)
        torch.cuda.synchronize()
        ref = (d_out.clone(), d_off.clone(), d_status.clone(), d_cnt.clone())
        K = 50
        t0 = time.perf_counter()
        for _ in range(K):
            rnd(stream)
        torch.cuda.synchronize()
        eager = (time.perf_counter() - t0) / K * 1e3
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            rnd(stream)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            g.replay()
        torch.cuda.synchronize()
        graph = (time.perf_counter() - t0) / K * 1e3
    same = all(torch.equal(a, b) for a, b in zip(ref, (d_out, d_off, d_status, d_cnt)))
    print(f"eager {eager:.4f} ms/round, graph replay {graph:.4f} ms/round, outputs identical: {same}", flush=True)


if __name__ == "__main__":
    main()
