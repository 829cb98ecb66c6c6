#!/usr/bin/env python3
"""In-process A/B of an interface-engine knob (the bench's nic leg: the C3
round's delivered events through every host's router + receive bucket),
alternating arms, outputs compared.  Usage: nic_probe.py ENV V1 V2 ..."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from shadow_amd import Topology, _lib, scenario, synth
    from shadow_amd.router import HEADER_UDP, Interfaces
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
    top.process_device(d_recs.data_ptr(), P, 110_000_000, 10**15, 0, d_out.data_ptr(), d_off.data_ptr(),
                       d_status.data_ptr(), d_cnt.data_ptr(), 0)
    n = int(d_off[-1].item())
    lib = _lib.lib()
    d_len = torch.empty(n, dtype=torch.int32, device=dev)
    _lib.check(lib.shd_event_lengths(d_out.data_ptr(), n, d_recs.data_ptr(), HEADER_UDP, d_len.data_ptr(), None))
    tmax = int(d_out.view(torch.int64).view(-1, 4)[:n, 0].max().item())
    gbit = 1_000_000_000 // 8 // 1024
    bw = np.full(H, gbit, dtype=np.uint64)
    nic = Interfaces(H, bw, bw, 100_000_000, 4096, n, device=dev)
    s0 = nic.states.clone()
    name, vals = sys.argv[1], sys.argv[2:]
    outs = {}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rep in range(3):
        for v in vals:
            if v == "-":
                os.environ.pop(name, None)
            else:
                os.environ[name] = v
            ms = []
            for r in range(6):
                nic.states.copy_(s0)
                torch.cuda.synchronize()
                e0.record()
                nic.run_device(d_out.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), tmax + 1)
                e1.record()
                torch.cuda.synchronize()
                if r:
                    ms.append(e0.elapsed_time(e1))
            print(f"{name}={v} rep {rep}: shd_nic_run {np.median(ms):.4f} ms (median of 5)", flush=True)
            outs[v] = (nic.recv_time.clone(), nic.recv_status.clone(), nic.states.clone(), nic.rings.clone())
    same = all(all(torch.equal(a, b) for a, b in zip(outs[vals[0]], outs[v])) for v in vals[1:])
    print(f"outputs identical: {same}", flush=True)


if __name__ == "__main__":
    main()
