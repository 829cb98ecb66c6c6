#!/usr/bin/env python3
"""Where a C3 round's wall time goes besides its kernels (dev tool): 50
rounds of shd_round_process_device on one stream, the host's time to issue
them (before the sync) and the total, with the per-stage timing events off
and on."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from shadow_amd import Topology, _lib, scenario, synth
    lib = _lib.lib()
    V, H, P = 20_000, 100_000, 10_000_000
    top = Topology(synth.sparse_graph_gml(V, 0x5EED0002))
    ips, st, verts = scenario.register_hosts(top, H, seed=1)
    A = top.slot_count()
    tab = torch.empty(A * A * 2, dtype=torch.float64, device="cuda")
    top.build_rows_device(0, A, tab.data_ptr())
    torch.cuda.synchronize()
    top.adopt_table_device_resident(tab.data_ptr())
    top.touch_all()
    pk = synth.packet_batch(P, H, 0x5EED0003, 100_000_000, 10_000_000, st)
    d_recs = torch.from_numpy(pk.view(np.uint8)).cuda()
    out = torch.empty(P * 32, dtype=torch.uint8, device="cuda")
    off = torch.empty(H + 1, dtype=torch.int32, device="cuda")
    status = torch.empty(P, dtype=torch.uint8, device="cuda")
    cnt = torch.empty(2, dtype=torch.int64, device="cuda")
    stream = torch.cuda.Stream()
    sp = stream.cuda_stream

    def rnd():
        top.process_device(d_recs.data_ptr(), P, 110_000_000, 10**15, 0, out.data_ptr(), off.data_ptr(),
                           status.data_ptr(), cnt.data_ptr(), sp)

    for _ in range(5):
        rnd()
    torch.cuda.synchronize()
    K = 50
    for timing in (0, 1, 0, 1):
        _lib.check(lib.shd_round_timing_enable(timing))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        per = []
        for _ in range(K):
            a = time.perf_counter()
            rnd()
            per.append(time.perf_counter() - a)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        per.sort()
        print(f"timing={timing}: {(t2 - t0) / K * 1e3:.3f} ms/round; host issue {(t1 - t0) / K * 1e3:.3f} ms/round "
              f"(median call {per[K // 2] * 1e3:.3f} ms, max {per[-1] * 1e3:.3f} ms)", flush=True)
        _lib.check(lib.shd_round_timing_enable(0))
    top.close()


if __name__ == "__main__":
    main()
