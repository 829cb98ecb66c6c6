"""C4 rounds as a simulation, not a replay.

On the C4 graph (configs[4]: V = 100k, H = 200k; the 120 GB table
device-resident, every row released in slot order -- the steady state the
first round leads to), three rounds of the device load generator
(shd_synth_sends_device) and the hand-off: the barrier advances by the
window every round, every sender's rand_r state and event counter are
carried on the device from round to round (one reserved draw per packet,
worker.c:540-541), and the destinations are new every round.  Senders and
destinations are a sampled pool of hosts, so that the oracle computes only
their rows (igraph-0.8 Dijkstra restatement, independent of the GPU table).
Per round: the generated records bit for bit against the numpy restatement
(synth.synth_sends) with the states carried on the host, and the decided
round -- statuses, events in event_compare order, minimum time -- against the
oracle; at the end the carried states against the host's."""
import ctypes as C
import time

import numpy as np
import pytest

import count_check
import oracle_ctypes as O
from shadow_amd import Topology, _lib, scenario, synth

pytestmark = pytest.mark.gpu

V4, H4 = 100_000, 200_000
SEED, M, W, T0, END = 0x5EED0C40, 4, 10_000_000, 100_000_000, 10**15


def progress(t0, *a):
    print(f"[c4sim {time.perf_counter() - t0:7.1f}s]", *a, flush=True)


@pytest.mark.timeout(60)
def test_c4_three_simulated_rounds():
    import torch
    t_start = time.perf_counter()
    gml = synth.sparse_graph_gml(V4, 0x5EED0004)  # the bench's C4 graph
    top = Topology(gml)
    ips, st, verts = scenario.register_hosts(top, H4, seed=1)
    A = top.slot_count()
    table = top.alloc_table(A * A * 16)
    top.build_rows_device(0, A, table.ptr)
    torch.cuda.synchronize()
    top.adopt_table_device_resident(table.ptr)
    top.touch_all()
    progress(t_start, f"C4 table A={A} built, adopted, every row released")
    pool = np.unique(np.random.default_rng(0x5EED0C41).integers(0, H4, 256)).astype(np.uint32)
    npool = len(pool)
    orc = O.OracleTopology(gml)
    ips2, st2, verts2 = scenario.register_hosts(orc, H4, seed=1)
    assert (st2 == st).all() and (verts2 == verts).all()
    sv = np.unique(verts[pool]).astype(np.int32)  # ascending vertex = ascending slot = touch order
    lat, rel = orc.rows_parallel(sv, sv, 16)
    orc.preload(sv, lat, rel)
    progress(t_start, f"oracle rows of the {len(sv)} pool vertices")
    lib = _lib.lib()
    dev = torch.device("cuda")
    d_pool = torch.from_numpy(pool.view(np.int32)).to(dev)
    d_st = [torch.from_numpy(st[pool].astype(np.uint32).view(np.int32)).to(dev), torch.empty(npool, dtype=torch.int32,
                                                                                             device=dev)]
    d_sq = [torch.zeros(npool, dtype=torch.int64, device=dev), torch.empty(npool, dtype=torch.int64, device=dev)]
    n = npool * M
    d_recs = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    d_out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    d_off = torch.empty(H4 + 1, dtype=torch.int32, device=dev)
    d_status = torch.empty(n, dtype=torch.uint8, device=dev)
    d_cnt = torch.empty(2, dtype=torch.int64, device=dev)
    h_states, h_seqs = st[pool].astype(np.uint32), np.zeros(npool, dtype=np.uint64)
    all_recs, all_status = [], []
    for r in range(3):
        t0, barrier = T0 + r * W, T0 + (r + 1) * W
        a, b = r % 2, (r + 1) % 2
        _lib.check(lib.shd_synth_sends_device(C.c_void_p(d_pool.data_ptr()), npool, M, r, SEED, t0, W,
                                              C.c_void_p(d_pool.data_ptr()), npool, C.c_void_p(d_st[a].data_ptr()),
                                              C.c_void_p(d_st[b].data_ptr()), C.c_void_p(d_sq[a].data_ptr()),
                                              C.c_void_p(d_sq[b].data_ptr()), C.c_void_p(d_recs.data_ptr()), None))
        top.process_device(d_recs.data_ptr(), n, barrier, END, 0, d_out.data_ptr(), d_off.data_ptr(),
                           d_status.data_ptr(), d_cnt.data_ptr(), 0)
        torch.cuda.synchronize()
        want, h_states, h_seqs = synth.synth_sends(pool, M, r, SEED, t0, W, h_states, h_seqs, dst_pool=pool)
        recs = d_recs.cpu().numpy().view(synth.PKT_DTYPE)
        assert recs.tobytes() == want.tobytes(), f"round {r}: generated records"
        cnt = d_cnt.cpu().numpy().view(np.uint64)
        out = d_out.cpu().numpy().view(synth.DELIV_DTYPE)[:cnt[0]]
        oout, ostatus, omt = orc.round(ips, recs, barrier, END)
        assert np.array_equal(d_status.cpu().numpy(), ostatus), f"round {r}: status"
        assert int(cnt[1]) == omt, f"round {r}: min time"
        assert np.array_equal(out, oout), f"round {r}: events"
        assert out["time"].min() >= barrier  # (inter-host deliveries clamp to the advancing barrier)
        all_recs.append(recs.copy())
        all_status.append(ostatus)
        progress(t_start, f"round {r}: {len(out)} of {n} delivered, equal to the oracle")
    # path packet counters accumulated over the three device rounds
    # (worker.c:551): every counter of the owner rows against the
    # restatement, every pool pair against the oracle's counters
    hslot = count_check.slot_map(verts)
    keys, counts = count_check.expected_keys(hslot, np.concatenate(all_recs), np.concatenate(all_status), A)
    count_check.check_rows(top, keys, counts, A, np.unique(keys // A))
    for x in pool:
        for y in pool[::7]:
            assert top.path_packet_count(int(ips[x]), int(ips[y])) == orc.packet_count(int(ips[x]), int(ips[y]))
    progress(t_start, f"path packet counters of {len(np.unique(keys // A))} rows equal")
    assert np.array_equal(d_st[1].cpu().numpy().view(np.uint32), h_states)  # (3 rounds: the carry ends in [1])
    assert np.array_equal(d_sq[1].cpu().numpy().view(np.uint64), h_seqs)
    top.close()
    orc.close()
    del table
    torch.cuda.empty_cache()


def test_synth_sends_rejects_overlapping_carry():
    """The load generator's carried states: in and out arrays that overlap
    (for the rand_r states or the event counters) are refused (-EINVAL)."""
    import torch
    lib = _lib.lib()
    dev = torch.device("cuda")
    npool, m = 64, 4
    pool = torch.arange(npool, dtype=torch.int32, device=dev)
    st = torch.zeros(2 * npool, dtype=torch.int32, device=dev)
    sq = torch.zeros(2 * npool, dtype=torch.int64, device=dev)
    recs = torch.empty(npool * m * 32, dtype=torch.uint8, device=dev)
    P = lambda t, off=0: C.c_void_p(t.data_ptr() + off * t.element_size())  # noqa: E731

    def call(st_in, st_out, sq_in, sq_out):
        return lib.shd_synth_sends_device(P(pool), npool, m, 0, 1, 0, 1000, None, 1000, st_in, st_out, sq_in, sq_out,
                                          P(recs), None)
    assert call(P(st), P(st, npool), P(sq), P(sq, npool)) == 0
    torch.cuda.synchronize()
    assert call(P(st), P(st, npool), P(sq), P(sq)) == -22           # the same counters
    assert call(P(st), P(st, npool), P(sq), P(sq, npool // 2)) == -22  # overlapping counters
    assert call(P(st), P(st, 1), P(sq), P(sq, npool)) == -22           # overlapping states
