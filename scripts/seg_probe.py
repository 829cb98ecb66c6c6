#!/usr/bin/env python3
"""The decided round at the destination-segment sizes an owner sees at N
ranks (dev tool): 10M packets per round over H hosts on the V = 20k graph,
H = 100k (C3: ~92 events per destination) and H = 100k / N (the ~92 N
events per destination of a weak-scaled N-rank exchange, whose owner holds
100k / N hosts).  Per H: ms per round and the stage times, per pipeline
knob value given.  Usage: seg_probe.py [ENV VALUE ...]"""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from shadow_amd import Topology, _lib, scenario, synth
    env = sys.argv[1] if len(sys.argv) > 1 else None
    vals = sys.argv[2:] if env else [None]
    lib = _lib.lib()
    P = 10_000_000
    for H in (100_000, 25_000, 12_500):
        top = Topology(synth.sparse_graph_gml(20_000, 0x5EED0002))
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
        for v in vals:
            if env:
                os.environ[env] = v
            top.process_device(d_recs.data_ptr(), P, 110_000_000, 10**15, 0, out.data_ptr(), off.data_ptr(),
                               status.data_ptr(), cnt.data_ptr(), 0)
            torch.cuda.synchronize()
            _lib.check(lib.shd_round_timing_enable(1))
            t0 = time.perf_counter()
            for _ in range(10):
                top.process_device(d_recs.data_ptr(), P, 110_000_000, 10**15, 0, out.data_ptr(), off.data_ptr(),
                                   status.data_ptr(), cnt.data_ptr(), 0)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 10 * 1e3
            st_ms = (C.c_double * 4)()
            nl = C.c_int()
            _lib.check(lib.shd_round_timing_read(st_ms, 4, C.byref(nl)))
            _lib.check(lib.shd_round_timing_enable(0))
            k = max(nl.value, 1)
            print(f"H={H} ({P / H:.0f} per destination) {env}={v}: {dt:.3f} ms/round; stages "
                  + " ".join(f"{st_ms[i] / k:.4f}" for i in range(4)), flush=True)
        del tab, d_recs, out
        top.close()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
