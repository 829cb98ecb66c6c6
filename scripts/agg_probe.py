#!/usr/bin/env python3
"""In-process A/B of a per-launch knob on the C3 round (no allocation / box
variance between the arms): alternating blocks of 20 rounds, live per-stage
timing, outputs compared.  Usage: agg_probe.py [ENV_NAME VALUE VALUE ...]
(default: SHD_DEST_AGG 1 0); VALUE "-" leaves the variable unset."""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from shadow_amd import Topology, scenario, synth, _lib
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
    outs = {}

    def run_round():
        try:
            top.process_device(d_recs.data_ptr(), P, 110_000_000, 10**15, 0, d_out.data_ptr(),
                               d_off.data_ptr(), d_status.data_ptr(), d_cnt.data_ptr(), 0)
        except _lib.ShdError:
            # a measurement-only arm (SHD_SCATTER_PROBE) skips stores on purpose: the
            # round's guards fire (-EIO for that round); its timing still counts
            if name != "SHD_SCATTER_PROBE":
                raise
    name, vals = (sys.argv[1], sys.argv[2:]) if len(sys.argv) > 2 else ("SHD_DEST_AGG", ["1", "0"])
    for rep in range(3):
        for agg in vals:
            if agg == "-":
                os.environ.pop(name, None)
            else:
                os.environ[name] = agg
            for _ in range(2):
                run_round()
            if os.environ.get("PROBE_SYNC_COUNTS") == "1":
                top.path_counts_sync()  # (the warm-up rounds' counts: outside the timed block)
            torch.cuda.synchronize()
            _lib.check(lib.shd_round_timing_enable(1))
            t0 = time.perf_counter()
            for _ in range(20):
                run_round()
            if os.environ.get("PROBE_SYNC_COUNTS") == "1":  # the logged path counts folded in the timed block
                top.path_counts_sync()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 20 * 1e3
            st = (C.c_double * 4)()
            nl = C.c_int()
            _lib.check(lib.shd_round_timing_read(st, 4, C.byref(nl)))
            _lib.check(lib.shd_round_timing_enable(0))
            k = max(nl.value, 1)
            print(f"{name}={agg} rep {rep}: round {dt:.4f} ms, scatter {st[0] / k:.4f} ms, scan {st[1] / k:.4f}, "
                  f"place {st[2] / k:.4f}, sort {st[3] / k:.4f} ms", flush=True)
            outs[agg] = (d_out.clone(), d_off.clone(), d_status.clone())
    same = all(all(torch.equal(a, b) for a, b in zip(outs[vals[0]], outs[v])) for v in vals[1:])
    print(f"outputs identical: {same}", flush=True)


if __name__ == "__main__":
    main()
