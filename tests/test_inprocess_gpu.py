"""Multi-rank rounds with the ranks as threads of ONE process (Shadow runs
one process with one manager, core/manager.c:543-577): one topology and one
thread per rank, the in-process transport (shd_transport_local_new: a thread
barrier plus device-to-device copies), all ranks on GPU 0 here.  Each rank
builds its share of the rows, the C-ABI all-gather completes every rank's
table, then each rank decides its senders' packets and the events go to
their destinations' owners -- both with shd_round_process_exchange (grouped,
24-B wire records) and with shd_round_process_device + shd_round_exchange.
The union over ranks must equal the oracle's single round."""
import threading

import numpy as np
import pytest

import oracle_ctypes as O

pytestmark = pytest.mark.gpu

H = 300
BARRIER, END = 110_000_000, 10**15


def _gml():
    from shadow_amd import synth
    return synth.sparse_graph_gml(250, 0x5EED0801, ns_variant=True)


def _packets(rank, world, st):
    from shadow_amd import synth
    lo, hi = rank * H // world, (rank + 1) * H // world
    return synth.packet_batch(4000, H, 0x5EED0810 + rank, 100_000_000, 10_000_000, st, hosts_lo=lo, hosts_hi=hi)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("fused", [True, False], ids=["process_exchange", "device+exchange"])
def test_threads_as_ranks(world, fused):
    import torch

    from shadow_amd import Topology, scenario, synth
    from shadow_amd.transport import InProcessTransports
    xps = InProcessTransports(world, "local")
    tops, res, errs = [], [None] * world, []
    gml = _gml()
    for r in range(world):
        top = Topology(gml)
        ips, st, verts = scenario.register_hosts(top, H, seed=1)
        tops.append((top, st))
    A = tops[0][0].slot_count()
    row_bounds = [r * A // world for r in range(world + 1)]
    host_bounds = [r * H // world for r in range(world + 1)]
    bufs = []
    for r in range(world):
        n = 4000
        cap = n * world
        bufs.append(dict(
            tab=torch.zeros(A * A * 2, dtype=torch.float64, device="cuda"),
            recs=torch.from_numpy(_packets(r, world, tops[r][1]).view(np.uint8)).cuda(),
            send=torch.empty(n * 32, dtype=torch.uint8, device="cuda"),
            off=torch.empty(H + 1, dtype=torch.int32, device="cuda"),
            status=torch.empty(n, dtype=torch.uint8, device="cuda"),
            cnt=torch.empty(2, dtype=torch.int64, device="cuda"),
            recv=torch.empty(cap * 32, dtype=torch.uint8, device="cuda"),
            fin=torch.empty(cap * 32, dtype=torch.uint8, device="cuda"),
            fin_off=torch.empty(host_bounds[r + 1] - host_bounds[r] + 1, dtype=torch.int32, device="cuda")))
    torch.cuda.synchronize()

    def rank_main(r):
        try:
            top, _ = tops[r]
            b, xp = bufs[r], xps.ranks[r]
            lo, hi = row_bounds[r], row_bounds[r + 1]
            if hi > lo:
                top.build_rows_device(lo, hi, b["tab"].data_ptr())
            top.allgather_rows(xp, b["tab"].data_ptr(), row_bounds)
            top.adopt_table_device(b["tab"].data_ptr())
            top.touch_all()
            n = 4000
            if fused:
                nrecv = top.process_exchange(xp, b["recs"].data_ptr(), n, BARRIER, END, 0, host_bounds,
                                             b["send"].data_ptr(), b["status"].data_ptr(), b["cnt"].data_ptr(),
                                             b["recv"].data_ptr(), n * world, b["fin"].data_ptr(),
                                             b["fin_off"].data_ptr())
            else:
                top.process_device(b["recs"].data_ptr(), n, BARRIER, END, 0, b["send"].data_ptr(),
                                   b["off"].data_ptr(), b["status"].data_ptr(), b["cnt"].data_ptr(), 0)
                nrecv = top.exchange(xp, b["send"].data_ptr(), b["off"].data_ptr(), host_bounds, b["recv"].data_ptr(),
                                     n * world, b["fin"].data_ptr(), b["fin_off"].data_ptr())
            res[r] = nrecv
        except BaseException as e:  # reported by the main thread
            errs.append(e)

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in th), "a rank thread is stuck in a collective"
    assert not errs, errs[0]
    xps.close()
    orc = O.OracleTopology(gml)
    ips, st, verts = scenario.register_hosts(orc, H, 1)
    sv = np.unique(verts).astype(np.int32)
    lat, rel = orc.rows_parallel(sv, sv, 8)
    want = np.stack([lat, rel], axis=-1).tobytes()
    for b in bufs:  # every rank's all-gathered table
        assert b["tab"].cpu().numpy().tobytes() == want
    orc.preload(sv, lat, rel)
    allpk = np.concatenate([_packets(r, world, st) for r in range(world)])
    ref, status, mt = orc.round(ips, allpk, BARRIER, END)
    merged = np.concatenate([bufs[r]["fin"].cpu().numpy().view(synth.DELIV_DTYPE)[:res[r]] for r in range(world)])
    assert len(merged) == len(ref)
    for k in ("dst_host", "time", "src_host", "seq"):
        assert np.array_equal(merged[k], ref[k]), k
    assert min(int(b["cnt"].cpu().numpy().view(np.uint64)[1]) for b in bufs) == mt
    for r in range(world):
        offs = bufs[r]["fin_off"].cpu().numpy()
        got = bufs[r]["fin"].cpu().numpy().view(synth.DELIV_DTYPE)[:res[r]]
        assert offs[-1] == res[r]
        assert np.array_equal(np.diff(offs), np.bincount(got["dst_host"] - host_bounds[r],
                                                         minlength=host_bounds[r + 1] - host_bounds[r]))
