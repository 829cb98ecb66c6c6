#!/usr/bin/env python3
"""In-process A/B of a knob of the interface engine (shd_nic_run) on the C3
round's output, as bench.py's nic leg runs it: alternating blocks of 10
windows, HIP events on the launch stream, fates compared between arms.
Usage: nic_probe.py ENV_NAME VALUE VALUE ...  (VALUE "-": unset)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from shadow_amd import Topology, scenario, synth, _lib
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
    torch.cuda.synchronize()
    delivered = int(d_off[H].item())
    lib = _lib.lib()
    stream = torch.cuda.Stream(dev)
    sptr = stream.cuda_stream
    d_len = torch.empty(max(delivered, 1), dtype=torch.int32, device=dev)
    _lib.check(lib.shd_event_lengths(d_out.data_ptr(), delivered, d_recs.data_ptr(), HEADER_UDP, d_len.data_ptr(),
                                     sptr))
    tmax = int(d_out.view(torch.int64).view(-1, 4)[:delivered, 0].max().item())
    gbit = 1_000_000_000 // 8 // 1024
    bw = np.full(H, gbit, dtype=np.uint64)
    nic = Interfaces(H, bw, bw, 100_000_000, 4096, max(delivered, 1), device=dev)
    states0 = nic.states.clone()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    name, vals = sys.argv[1], sys.argv[2:]
    fates = {}
    for rep in range(3):
        for v in vals:
            if v == "-":
                os.environ.pop(name, None)
            else:
                os.environ[name] = v
            ms = []
            for r in range(11):
                nic.states.copy_(states0)
                torch.cuda.synchronize(dev)
                ev0.record(stream)
                nic.run_device(d_out.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), tmax + 1, 0, 0, stream=sptr)
                ev1.record(stream)
                torch.cuda.synchronize(dev)
                if r:
                    ms.append(ev0.elapsed_time(ev1))
            t, st = nic.fates()
            fates[v] = (t.clone() if hasattr(t, "clone") else np.copy(t), st.clone() if hasattr(st, "clone") else
                        np.copy(st), nic.states.clone(), nic.rings.clone())
            print(f"{name}={v} rep {rep}: window {np.mean(ms):.4f} ms (min {min(ms):.4f})", flush=True)
    ref = fates[vals[0]]
    same = True
    for v in vals[1:]:
        for a, b in zip(ref, fates[v]):
            same &= bool((a == b).all()) if hasattr(a, "all") else a == b
    print(f"fates and states identical: {same}", flush=True)


if __name__ == "__main__":
    main()
