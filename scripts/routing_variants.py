#!/usr/bin/env python3
"""Times the slab routing kernel's measurement variants (same exact
algorithm: SHD_SSSP_TOP = LDS heap positions per wave, SHD_SSSP_WAVES) on
the C2 (and optionally C4) build and checks every variant's table is bitwise
equal to the first one's.  Usage: routing_variants.py [--c4] VARIANT...
VARIANT = "kern=islab|blk|slab[,top=256|512][,wpe=7|8][,waves=N]" (islab: the
integer-key blocked heap, whole-ms graphs)."""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c4", action="store_true")
    ap.add_argument("--c1", action="store_true", help="the C1 complete graph (LDS kernel) instead of C2")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    import torch

    from shadow_amd import Topology, scenario, synth
    cfgs = ([("C1", 1000, 5000, 0x5EED0001)] if a.c1 else [("C2", 20_000, 100_000, 0x5EED0002)]) + \
        ([("C4", 100_000, 200_000, 0x5EED0004)] if a.c4 else [])
    for name, V, H, seed in cfgs:
        gml = synth.complete_graph_gml(V, seed) if name == "C1" else synth.sparse_graph_gml(V, seed)
        top = Topology(gml)
        scenario.register_hosts(top, H, seed=1)
        A = top.slot_count()
        ref = None
        tab = torch.empty(A * A * 2, dtype=torch.float64, device="cuda")
        for v in a.variants:
            kv = dict(x.split("=") for x in v.split(","))
            os.environ["SHD_SSSP_TOP"] = kv.get("top", "256")
            os.environ["SHD_SSSP_KERNEL"] = kv.get("kern", "islab")
            os.environ["SHD_SSSP_WPE"] = kv.get("wpe", "8")
            os.environ["SHD_SSSP_LDS_SEQ"] = kv.get("seq", "0")
            if "waves" in kv:
                os.environ["SHD_SSSP_WAVES"] = kv["waves"]
            else:
                os.environ.pop("SHD_SSSP_WAVES", None)
            ts = []
            for _ in range(a.reps if name != "C4" else 1):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                top.build_rows_device(0, A, tab.data_ptr())
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            # checksum of the table bits (a full copy of C4 is 120 GB)
            h = tab.view(torch.int64)
            sig = (int(h[::997].sum().item()), int(h[1::1009].sum().item()), int((h[: A * 2 * 64]).sum().item()))
            if ref is None:
                ref = sig
            print(f"{name} {v}: {min(ts):.5f}s (all {', '.join(f'{t:.5f}' for t in ts)}) "
                  f"{'same' if sig == ref else 'DIFFERENT'}", flush=True)
            if sig != ref:
                sys.exit(1)
        del tab
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
