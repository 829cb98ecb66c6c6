"""Timing probe at config scale (dev tool): C1 and C2 routing builds and one
10M-packet round.  Prints one line per measurement."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from shadow_amd import Topology, scenario, synth  # noqa: E402


def timed(label, fn):
    t0 = time.perf_counter()
    r = fn()
    print(f"{label}: {time.perf_counter() - t0:.3f} s", flush=True)
    return r


def main():
    which = sys.argv[1:] or ["c1", "c2", "c3"]
    if "c1" in which:
        gml = timed("c1 gen", lambda: synth.complete_graph_gml(1000, 0x5EED0001))
        top = timed("c1 load", lambda: Topology(gml))
        timed("c1 attach 5000", lambda: scenario.register_hosts(top, 5000))
        timed("c1 build (incl. upload + mirror)", top.build_routes)
        A = top.slot_count()
        tab = torch.empty(A * A * 2, dtype=torch.float64, device="cuda")
        for r in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            top.build_rows_device(0, A, tab.data_ptr())
            torch.cuda.synchronize()
            print(f"c1 rows kernel A={A}: {time.perf_counter() - t0:.4f} s", flush=True)
    if "c2" in which or "c3" in which:
        V = int(os.environ.get("PROBE_V", "20000"))
        H = int(os.environ.get("PROBE_H", "100000"))
        gml = timed("c2 gen", lambda: synth.sparse_graph_gml(V, 0x5EED0002))
        top = timed("c2 load", lambda: Topology(gml))
        ips, st, _ = timed(f"c2 attach {H}", lambda: scenario.register_hosts(top, H))
        A = top.slot_count()
        print("A =", A, flush=True)
        tab = torch.empty(A * A * 2, dtype=torch.float64, device="cuda")
        rows = int(os.environ.get("PROBE_ROWS", "2048"))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        top.build_rows_device(0, min(rows, A), tab.data_ptr())
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"c2 rows kernel {min(rows, A)} rows: {dt:.3f} s -> full table est {dt * A / min(rows, A):.1f} s",
              flush=True)
        if "c3" in which and rows >= A:
            timed("adopt (mirror D2H)", lambda: top.adopt_table_device(tab.data_ptr()))
            timed("touch_all", top.touch_all)
            pk = timed("gen 10M packets", lambda: synth.packet_batch(10_000_000, H, 0x5EED0003, 100_000_000,
                                                                      10_000_000, st))
            n = len(pk)
            d_recs = torch.from_numpy(pk.view(np.uint8)).cuda()
            d_out = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
            d_off = torch.empty(H + 1, dtype=torch.int32, device="cuda")
            d_status = torch.empty(n, dtype=torch.uint8, device="cuda")
            d_cnt = torch.empty(2, dtype=torch.int64, device="cuda")
            for r in range(5):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                top.process_device(d_recs.data_ptr(), n, 110_000_000, 10**15, 0, d_out.data_ptr(), d_off.data_ptr(),
                                   d_status.data_ptr(), d_cnt.data_ptr(), 0)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                print(f"round {r}: {dt * 1e3:.3f} ms  {n / dt / 1e9:.3f} Gpkt/s", flush=True)
            print("delivered", d_cnt.cpu().numpy().view(np.uint64), flush=True)


if __name__ == "__main__":
    main()
