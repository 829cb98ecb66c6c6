#!/usr/bin/env python3
"""C3 rounds for a kernel trace of the round's launch sequence (gaps between
kernels): ROUND_TIMING=1 records the per-stage HIP events as bench.py does,
0 leaves them out (the product's synchronous call).  Usage, on the box:
rocprofv3 --kernel-trace -f csv -d DIR -o t -- python3 scripts/round_trace.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from shadow_amd import Topology, _lib, scenario, synth
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
    lib = _lib.lib()
    timing = os.environ.get("ROUND_TIMING", "1") == "1"
    for _ in range(3):
        top.process_device(d_recs.data_ptr(), P, 110_000_000, 10**15, 0, d_out.data_ptr(), d_off.data_ptr(),
                           d_status.data_ptr(), d_cnt.data_ptr(), 0)
    top.path_counts_sync()
    torch.cuda.synchronize()
    if timing:
        _lib.check(lib.shd_round_timing_enable(1))
    t0 = time.perf_counter()
    k = int(os.environ.get("ROUND_N", "10"))
    for _ in range(k):
        top.process_device(d_recs.data_ptr(), P, 110_000_000, 10**15, 0, d_out.data_ptr(), d_off.data_ptr(),
                           d_status.data_ptr(), d_cnt.data_ptr(), 0)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / k * 1e3
    if timing:
        _lib.check(lib.shd_round_timing_enable(0))
    print(f"timing {int(timing)}: {dt:.4f} ms per round (wall, {k} rounds, counts not folded)", flush=True)


if __name__ == "__main__":
    main()
