#!/usr/bin/env python3
"""What the exchanged round costs on one GPU (dev tool): the C3 round (10M
packets over 100k hosts, V = 20k) as shd_round_process_device and as
shd_round_process_exchange over the library's RCCL transport to itself
(one rank: the decide, the grouped wire records, the count and payload
all-to-alls, the run merge) -- the N>1 step's fixed machinery without xGMI.
Alternating blocks of 10 rounds, wall clock with a device sync per block.

`xchg_probe.py local N`: N ranks as threads on the one GPU over the local
transport, 10M packets per rank (senders: the rank's own hosts) over the
same 100k hosts -- the owner's segments of ~92 N events from N runs of a
weak-scaled exchange; ms per exchanged round (all N ranks, serialised on the
one GPU) with SHD_WIRE_SORTED unset (the default rule), 1 and 0, and the
unions checked equal; each rank's phase times of its last split exchange
(shd_round_exchange_phases).  XCHG_PROBE_KNOB=SHD_XCHG_SPLIT=1/0: the split
exchange against one group after the whole round."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def local_ranks(N):
    import threading

    import torch

    from shadow_amd import Topology, scenario, synth
    from shadow_amd.transport import InProcessTransports
    V, H, P = 20_000, 100_000, 10_000_000
    gml = synth.sparse_graph_gml(V, 0x5EED0002)
    tops, sts = [], []
    for r in range(N):
        top = Topology(gml)
        ips, st, verts = scenario.register_hosts(top, H, seed=1)
        tops.append(top)
        sts.append(st)
    A = tops[0].slot_count()
    tab = torch.empty(A * A * 2, dtype=torch.float64, device="cuda")
    tops[0].build_rows_device(0, A, tab.data_ptr())
    torch.cuda.synchronize()
    bounds = [r * H // N for r in range(N + 1)]
    bufs = []
    for r in range(N):
        tops[r].adopt_table_device_resident(tab.data_ptr())
        tops[r].touch_all()
        pk = synth.packet_batch(P, H, 0x5EED0003 + r, 100_000_000, 10_000_000, sts[r], hosts_lo=bounds[r],
                                hosts_hi=bounds[r + 1])
        bufs.append(dict(recs=torch.from_numpy(pk.view(np.uint8)).cuda(),
                         send=torch.empty(P * 32, dtype=torch.uint8, device="cuda"),
                         status=torch.empty(P, dtype=torch.uint8, device="cuda"),
                         cnt=torch.empty(2, dtype=torch.int64, device="cuda"),
                         recv=torch.empty(2 * P * 32, dtype=torch.uint8, device="cuda"),
                         fin=torch.empty(2 * P * 32, dtype=torch.uint8, device="cuda"),
                         fin_off=torch.empty(bounds[r + 1] - bounds[r] + 1, dtype=torch.int32, device="cuda")))
    torch.cuda.synchronize()
    xps = InProcessTransports(N, "local")
    nres = [0] * N
    errs = []
    phases = [None] * N
    import ctypes as C

    from shadow_amd import _lib

    def one(r, k):
        try:
            b = bufs[r]
            for _ in range(k):
                nres[r] = tops[r].process_exchange(xps.ranks[r], b["recs"].data_ptr(), P, 110_000_000, 10**15, 0,
                                                   bounds, b["send"].data_ptr(), b["status"].data_ptr(),
                                                   b["cnt"].data_ptr(), b["recv"].data_ptr(), 2 * P,
                                                   b["fin"].data_ptr(), b["fin_off"].data_ptr())
            # this thread's last split exchange (HIP events): decide, counts,
            # group 1, group 2, merge, whole call, transfer beside the decide
            ph = (C.c_double * 8)()
            ok = C.c_int()
            _lib.check(_lib.lib().shd_round_exchange_phases(ph, 8, C.byref(ok)))
            phases[r] = list(ph) if ok.value else None
        except BaseException as e:
            errs.append(e)

    def rounds(k):
        th = [threading.Thread(target=one, args=(r, k)) for r in range(N)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=300)
        assert not errs, errs
        torch.cuda.synchronize()

    def union():
        return np.concatenate([bufs[r]["fin"].cpu().numpy().view(synth.DELIV_DTYPE)[:nres[r]] for r in range(N)])

    try:
        outs = {}
        knob = os.environ.get("XCHG_PROBE_KNOB")  # NAME=v1/v2/...: A/B of another knob instead
        arms = ("auto", "1", "0", "auto", "1", "0")
        if knob:
            kn, kv = knob.split("=")
            arms = tuple(kv.split("/")) * 2
        for v in arms:
            if knob:
                os.environ[kn] = v
            elif v == "auto":
                os.environ.pop("SHD_WIRE_SORTED", None)
            else:
                os.environ["SHD_WIRE_SORTED"] = v
            rounds(1)
            t0 = time.perf_counter()
            rounds(5)
            dt = (time.perf_counter() - t0) / 5 * 1e3
            print(f"N={N} {knob.split('=')[0] if knob else 'SHD_WIRE_SORTED'}={v}: {dt:.3f} ms per exchanged round "
                  "(all ranks on one GPU), "
                  f"{sum(nres)} events", flush=True)
            for r in range(N):
                if phases[r]:
                    p = phases[r]
                    print(f"  rank {r}: decide {p[0]:.3f} counts {p[1]:.3f} group1 {p[2]:.3f} group2 {p[3]:.3f} "
                          f"merge {p[4]:.3f} call {p[5]:.3f} transfer beside decide {p[6]:.3f} "
                          f"merge beside group2 {p[7]:.3f} ms", flush=True)
            outs[v] = union()
        if not knob:
            print("sorted and unsorted wire unions identical:",
                  bool(np.array_equal(outs["1"], outs["0"]) and np.array_equal(outs["auto"], outs["0"])), flush=True)
    finally:
        xps.close()
        for t in tops:
            t.close()


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "local":
        return local_ranks(int(sys.argv[2]))
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
