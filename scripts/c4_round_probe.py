#!/usr/bin/env python3
"""Where a C4 round's time goes (dev tool): the C4 table (V = 100k, H = 200k,
120 GB) built, adopted device-resident and every row released, then blocks
of R rounds of 1M packets (200k senders x 5, the bench's C4 load) per arm,
alternating arms: new destinations every round ("sim") or one batch replayed
("replay"), by pipeline and table form (SHD_PTAB=0: the 16-B f64 entries;
else the 8-B packet-path copy).  Per arm: ms per round (wall, synchronised)
and the stage times (HIP events).
Usage: c4_round_probe.py [ARM ...]  ARM = mode:pipeline:ptab, e.g. sim:part:1"""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from shadow_amd import Topology, _lib, scenario, synth
    arms = sys.argv[1:] or ["sim:part:1", "replay:part:1", "sim:slab:1", "sim:part:0"]
    V4, H4, R = 100_000, 200_000, 20
    t0 = time.perf_counter()
    top = Topology(synth.sparse_graph_gml(V4, 0x5EED0004))
    ips, st, verts = scenario.register_hosts(top, H4, seed=1)
    A = top.slot_count()
    table = top.alloc_table(A * A * 16)
    top.build_rows_device(0, A, table.ptr)
    torch.cuda.synchronize()
    top.adopt_table_device_resident(table.ptr)
    top.touch_all()
    print(f"C4 table A={A} ready in {time.perf_counter() - t0:.1f}s", flush=True)
    lib = _lib.lib()
    dev = torch.device("cuda")
    pool = np.arange(H4, dtype=np.uint32)
    m, n = 5, H4 * 5
    d_pool = torch.from_numpy(pool.view(np.int32)).to(dev)
    d_st = [torch.from_numpy(st.astype(np.uint32).view(np.int32)).to(dev), torch.empty(H4, dtype=torch.int32,
                                                                                       device=dev)]
    d_sq = [torch.zeros(H4, dtype=torch.int64, device=dev), torch.empty(H4, dtype=torch.int64, device=dev)]
    d_recs = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    d_out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    d_off = torch.empty(H4 + 1, dtype=torch.int32, device=dev)
    d_status = torch.empty(n, dtype=torch.uint8, device=dev)
    d_cnt = torch.empty(2, dtype=torch.int64, device=dev)
    W, T0, END = 10_000_000, 100_000_000, 10**15
    rnd = [0]

    def gen():
        r = rnd[0]
        rnd[0] += 1
        a, b = r % 2, (r + 1) % 2
        _lib.check(lib.shd_synth_sends_device(C.c_void_p(d_pool.data_ptr()), H4, m, r, 0x5EED0008, T0 + r * W, W,
                                              None, H4, C.c_void_p(d_st[a].data_ptr()),
                                              C.c_void_p(d_st[b].data_ptr()), C.c_void_p(d_sq[a].data_ptr()),
                                              C.c_void_p(d_sq[b].data_ptr()), C.c_void_p(d_recs.data_ptr()), None))
        return T0 + (r + 1) * W

    def arm(spec):
        mode, pipe, ptab = spec.split(":")
        os.environ["SHD_PACKET_PIPELINE"] = pipe
        os.environ["SHD_PTAB"] = ptab
        barrier = gen()
        top.process_device(d_recs.data_ptr(), n, barrier, END, 0, d_out.data_ptr(), d_off.data_ptr(),
                           d_status.data_ptr(), d_cnt.data_ptr(), 0)
        torch.cuda.synchronize()
        _lib.check(lib.shd_round_timing_enable(1))
        s0 = time.perf_counter()
        for _ in range(R):
            if mode == "sim":
                barrier = gen()
            top.process_device(d_recs.data_ptr(), n, barrier, END, 0, d_out.data_ptr(), d_off.data_ptr(),
                               d_status.data_ptr(), d_cnt.data_ptr(), 0)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - s0) / R * 1e3
        st_ms = (C.c_double * 4)()
        nl = C.c_int()
        _lib.check(lib.shd_round_timing_read(st_ms, 4, C.byref(nl)))
        _lib.check(lib.shd_round_timing_enable(0))
        k = max(nl.value, 1)
        print(f"{spec}: {dt:.3f} ms/round (incl. generator for sim); stages "
              + " ".join(f"{st_ms[i] / k:.4f}" for i in range(4)) + " ms", flush=True)

    for rep in range(2):
        for a in arms:
            arm(a)
    top.close()


if __name__ == "__main__":
    main()
