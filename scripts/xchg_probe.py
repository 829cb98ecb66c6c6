#!/usr/bin/env python3
"""What the exchanged round costs on one GPU (dev tool): the C3 round (10M
packets over 100k hosts, V = 20k) as shd_round_process_device and as
shd_round_process_exchange over the library's RCCL transport to itself
(one rank: the decide, the grouped wire records, the count and payload
all-to-alls, the run merge) -- the N>1 step's fixed machinery without xGMI.
Alternating blocks of 10 rounds, wall clock with a device sync per block."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from shadow_amd import Topology, scenario, synth
    from shadow_amd.transport import InProcessTransports
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
    recv = torch.empty(P * 32, dtype=torch.uint8, device="cuda")
    fin = torch.empty(P * 32, dtype=torch.uint8, device="cuda")
    fin_off = torch.empty(H + 1, dtype=torch.int32, device="cuda")
    xps = InProcessTransports(1, "rccl", devices=[0])
    xp = xps.ranks[0]
    barrier, end = 110_000_000, 10**15

    def dev_round():
        top.process_device(d_recs.data_ptr(), P, barrier, end, 0, out.data_ptr(), off.data_ptr(), status.data_ptr(),
                           cnt.data_ptr(), 0)

    def xchg_round():
        top.process_exchange(xp, d_recs.data_ptr(), P, barrier, end, 0, [0, H], out.data_ptr(), status.data_ptr(),
                             cnt.data_ptr(), recv.data_ptr(), P, fin.data_ptr(), fin_off.data_ptr())

    try:
        for f in (dev_round, xchg_round):
            f()
        torch.cuda.synchronize()
        for rep in range(3):
            for name, f in (("process_device", dev_round), ("process_exchange (RCCL to self)", xchg_round)):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(10):
                    f()
                torch.cuda.synchronize()
                print(f"{name} rep {rep}: {(time.perf_counter() - t0) / 10 * 1e3:.3f} ms/round", flush=True)
        a = out.cpu().numpy().view(synth.DELIV_DTYPE)[:int(cnt.cpu().numpy().view(np.uint64)[0])]
        dev_round()
        torch.cuda.synchronize()
        b = out.cpu().numpy().view(synth.DELIV_DTYPE)[:int(cnt.cpu().numpy().view(np.uint64)[0])]
        xchg_round()
        torch.cuda.synchronize()
        n = int(fin_off.cpu().numpy()[-1])
        c = fin.cpu().numpy().view(synth.DELIV_DTYPE)[:n]
        print("outputs identical:", bool(np.array_equal(b, c)), len(a), n, flush=True)
    finally:
        xps.close()
        top.close()


if __name__ == "__main__":
    main()
