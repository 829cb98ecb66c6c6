#!/usr/bin/env python3
"""Times shd_deliv_sort_device (the regroup after the multi-GPU exchange) on
10M synthetic events over a 100k-host range, per pipeline (SHD_PACKET_PIPELINE
is read per launch).  REGROUP_ZIPF=1: skewed destinations (the hottest host
receives ~1/ln(H) of the events).  Usage: python scripts/bench_regroup.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shadow_amd import Topology, scenario, synth  # noqa: E402

n, lo, hi = 10_000_000, 0, int(os.environ.get("REGROUP_HOSTS", "100000"))
rng = np.random.default_rng(5)
ev = np.zeros(n, dtype=synth.DELIV_DTYPE)
ev["time"] = 110_000_000 + rng.integers(0, 150_000_000, n)
if os.environ.get("REGROUP_ZIPF") == "1":  # destination skew: log-uniform ranks (~Zipf(1)), host 0 hottest
    ev["dst_host"] = lo + np.minimum(np.floor(np.power(hi - lo, rng.random(n))).astype(np.int64) - 1, hi - lo - 1)
else:
    ev["dst_host"] = rng.integers(lo, hi, n)
ev["src_host"] = rng.integers(0, 100_000, n)
ev["seq"] = np.arange(n)
ev["pkt_index"] = np.arange(n)
top = Topology(synth.complete_graph_gml(5, 3))
scenario.register_hosts(top, 5, 1)
d_in = torch.from_numpy(ev.view(np.uint8)).cuda()
d_out = torch.empty_like(d_in)
d_off = torch.empty(hi - lo + 1, dtype=torch.int32, device="cuda")
for pipe in os.environ.get("REGROUP_PIPES", "rank,slab,rank,slab").split(","):
    os.environ["SHD_PACKET_PIPELINE"] = pipe
    for _ in range(2):
        top.deliv_sort_device(d_in.data_ptr(), n, lo, hi, d_out.data_ptr(), d_off.data_ptr(), 0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    k = 20
    for _ in range(k):
        top.deliv_sort_device(d_in.data_ptr(), n, lo, hi, d_out.data_ptr(), d_off.data_ptr(), 0)
    torch.cuda.synchronize()
    print(f"{pipe}: {(time.perf_counter() - t0) / k * 1e3:.3f} ms per 10M-event regroup over {hi - lo} hosts"
          f"{' (zipf destinations)' if os.environ.get('REGROUP_ZIPF') == '1' else ''}",
          flush=True)
