"""GPU parity at BASELINE.json's full configuration sizes.

C1: the whole 1,000-vertex complete-graph table (996 x 996 attached slots,
H = 5,000), ms and ns edge variants, every row bitwise against the oracle's
igraph-0.8 Dijkstra restatement (topology.c:1578-1814), rows on a thread pool.
C2: the V = 20k sparse graph with H = 50k hosts (18,339 attached slots), ms
and ns edge variants: every row of the table bitwise against the oracle.
C3: 10M packets with uniform, unrestricted senders and destinations over all
100k hosts on the V = 20k table; the oracle holds the whole 19,870^2 table.
C4: the V = 100k / H = 200k table built device-resident (120 GB), 1,027
sampled full-length rows bitwise, and a device-resident round whose packets
span all 200k hosts, decided against rows the oracle holds
(worker.c:536-576).
"""
import numpy as np
import pytest

import count_check
import oracle_ctypes as O
from shadow_amd import Topology, scenario, synth

pytestmark = pytest.mark.gpu

BARRIER, END = 110_000_000, 10**15


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


def device_round(top, pk, H, barrier=BARRIER, end=END, boot=0):
    """One shd_round_process_device call on HBM-resident records."""
    import torch
    n = len(pk)
    d_recs = torch.from_numpy(pk.view(np.uint8)).cuda()
    d_out = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    d_off = torch.empty(H + 1, dtype=torch.int32, device="cuda")
    d_status = torch.empty(n, dtype=torch.uint8, device="cuda")
    d_cnt = torch.empty(2, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    top.process_device(d_recs.data_ptr(), n, barrier, end, boot, d_out.data_ptr(), d_off.data_ptr(),
                       d_status.data_ptr(), d_cnt.data_ptr(), 0)
    torch.cuda.synchronize()
    cnt = d_cnt.cpu().numpy().view(np.uint64)
    out = d_out.cpu().numpy().view(synth.DELIV_DTYPE)[:cnt[0]].copy()
    return out, d_off.cpu().numpy().astype(np.int64), d_status.cpu().numpy(), int(cnt[1])


@pytest.mark.timeout(60)
@pytest.mark.parametrize("ns", [False, True], ids=["ms", "ns"])
def test_c1_full_table_bit_exact(ns):
    """configs[1]: every row of the V=1000 / H=5000 complete-graph table (the
    LDS kernel with 16 batches of 64 incident edges in flight per pop)."""
    gml = synth.complete_graph_gml(1000, 0x5EED0001, ns_variant=ns)
    top = Topology(gml)
    ips, st, verts = scenario.register_hosts(top, 5000, seed=1)
    orc = O.OracleTopology(gml)
    _, st2, verts2 = scenario.register_hosts(orc, 5000, seed=1)
    assert (verts == verts2).all() and (st == st2).all()
    lat, rel, sv = top.table()
    assert len(sv) == 996
    olat, orel = orc.rows_parallel(sv, sv)
    bad = np.flatnonzero((bits(lat) != bits(olat)).any(1) | (bits(rel) != bits(orel)).any(1))
    assert len(bad) == 0, f"{len(bad)} rows differ, first {bad[:5]}"
    if not ns:  # whole-ms latencies: the min-plus Floyd-Warshall latencies too
        import torch
        d = torch.empty(996 * 996, dtype=torch.float64, device="cuda")
        top.latency_table_fw(d.data_ptr())
        assert np.array_equal(bits(d.cpu().numpy().reshape(996, 996)), bits(olat))


@pytest.mark.timeout(60)
@pytest.mark.parametrize("ns", [False, True], ids=["ms", "ns"])
def test_c2_full_table_bit_exact(ns):
    """configs[2]: the V = 20k sparse graph with 50k hosts; every one of the
    18,339 rows of the slab-kernel table against the oracle's Dijkstra
    (compared in blocks of 2,048 rows, oracle rows on 16 threads)."""
    import time

    import torch
    H, V = 50_000, 20_000
    gml = synth.sparse_graph_gml(V, 0x5EED0002, ns_variant=ns)
    top = Topology(gml)
    ips, st, verts = scenario.register_hosts(top, H, seed=1)
    A = top.slot_count()
    sv = np.unique(verts).astype(np.int32)
    assert len(sv) == A and A > 18_000
    full = torch.empty(A * A * 2, dtype=torch.float64, device="cuda")
    top.build_rows_device(0, A, full.data_ptr())
    torch.cuda.synchronize()
    orc = O.OracleTopology(gml)
    _, st2, verts2 = scenario.register_hosts(orc, H, seed=1)
    assert (verts == verts2).all() and (st == st2).all()
    t0 = time.perf_counter()
    bad = []
    for b in range(0, A, 2048):
        rows = np.arange(b, min(A, b + 2048))
        got = full.view(A, A, 2)[b:b + len(rows)].cpu().numpy()
        olat, orel = orc.rows_parallel(sv[rows], sv, 16)
        diff = (bits(got[:, :, 0]) != bits(olat)).any(1) | (bits(got[:, :, 1]) != bits(orel)).any(1)
        bad += [int(x) for x in rows[diff]]
        print(f"[c2] rows {b}..{b + len(rows)} of {A} compared ({time.perf_counter() - t0:.1f}s)", flush=True)
    assert not bad, f"{len(bad)} rows differ, first {bad[:8]}"
    if not ns:  # whole-ms: the frontier SSSP's latencies equal the table's, every row
        d = torch.empty(A * A, dtype=torch.float64, device="cuda")
        t1 = time.perf_counter()
        top.latency_rows_frontier(0, A, d.data_ptr())
        print(f"[c2] frontier latencies of all {A} rows in {time.perf_counter() - t1:.3f}s", flush=True)
        assert torch.equal(d.view(A, A), full.view(A, A, 2)[:, :, 0])
        del d
    del full
    torch.cuda.empty_cache()


@pytest.mark.timeout(60)
def test_c3_uniform_unrestricted_round_bit_exact(monkeypatch):
    """configs[3] at full size with the bench's own distribution: 10M packets,
    senders and destinations uniform over all 100k hosts (segments of ~92
    events: the k_segsort_dst register sort), the oracle holding all 19,870
    rows released in slot order.  Statuses, delivery times, order, segment
    offsets and the min delivered time must all be equal -- for the slab and
    the part pipelines (SHD_PACKET_PIPELINE)."""
    import torch
    H, V = 100_000, 20_000
    gml = synth.sparse_graph_gml(V, 0x5EED0002)
    top = Topology(gml)
    ips, st, verts = scenario.register_hosts(top, H, seed=1)
    A = top.slot_count()
    full = torch.empty(A * A * 2, dtype=torch.float64, device="cuda")
    top.build_rows_device(0, A, full.data_ptr())
    torch.cuda.synchronize()
    top.adopt_table_device_resident(full.data_ptr())
    top.touch_all()  # steady state: every row released, in slot order (the oracle's preload order)
    sv = np.unique(verts).astype(np.int32)
    assert len(sv) == A
    orc = O.OracleTopology(gml)
    ips_o, _, verts_o = scenario.register_hosts(orc, H, seed=1)
    assert (verts == verts_o).all()
    tab = full.view(A, A, 2).cpu().numpy()
    # this H = 100k table itself, every one of its 19,870 rows, against the
    # oracle's Dijkstra (topology.c:1578-1814) before it is preloaded
    import time
    t0 = time.perf_counter()
    bad = []
    for b in range(0, A, 2048):
        rows = np.arange(b, min(A, b + 2048))
        olat, orel = orc.rows_parallel(sv[rows], sv, 16)
        diff = (bits(tab[rows, :, 0]) != bits(olat)).any(1) | (bits(tab[rows, :, 1]) != bits(orel)).any(1)
        bad += [int(x) for x in rows[diff]]
        print(f"[c3] table rows {b}..{b + len(rows)} of {A} compared ({time.perf_counter() - t0:.1f}s)", flush=True)
    assert not bad, f"{len(bad)} rows differ, first {bad[:8]}"
    orc.preload(sv, tab[:, :, 0], tab[:, :, 1])
    del tab
    pk = synth.packet_batch(10_000_000, H, 0x5EED0003, 100_000_000, 10_000_000, st)  # the bench's batch
    oout, ostatus, omt = orc.round(ips_o, pk, BARRIER, END)
    pipes = ("slab", "part")
    for pipe in pipes:
        monkeypatch.setenv("SHD_PACKET_PIPELINE", pipe)
        out, offs, status, mt = device_round(top, pk, H)
        assert np.array_equal(status, ostatus), pipe
        assert mt == omt, pipe
        assert offs[-1] == len(out) == len(oout), pipe
        assert np.array_equal(np.diff(offs), np.bincount(oout["dst_host"], minlength=H)), pipe
        assert np.array_equal(out, oout), pipe
        assert np.diff(offs).max() < 256  # uniform: every segment on the register-sort path
        del out
    # path packet counters, counted by the device rounds (worker.c:551): all
    # 19,870^2 counters against the numpy restatement (both rounds counted),
    # and 20k host pairs against the oracle's own counters
    hslot = count_check.slot_map(verts)
    C = top.path_packet_counts()
    want = count_check.expected_counts(hslot, pk, ostatus, A)
    assert int(want.sum()) == int(np.isin(ostatus, count_check.KEPT).sum())
    assert np.array_equal(C, want * len(pipes))
    del want
    rng = np.random.default_rng(5)
    k = rng.integers(0, len(pk), 20_000)
    count_check.check_against_oracle(C // len(pipes), hslot, orc, ips_o, pk["src_host"][k], pk["dst_host"][k])


@pytest.fixture(scope="module")
def c4():
    """configs[4]: V=100k sparse graph, 200k hosts, whole table in HBM."""
    import torch
    H, V = 200_000, 100_000
    gml = synth.sparse_graph_gml(V, 0x5EED0004)
    top = Topology(gml)
    ips, st, verts = scenario.register_hosts(top, H, seed=1)
    A = top.slot_count()
    full = torch.empty(A * A * 2, dtype=torch.float64, device="cuda")
    top.build_rows_device(0, A, full.data_ptr())
    torch.cuda.synchronize()
    top.adopt_table_device_resident(full.data_ptr())
    top.touch_all()  # steady state (slot order); lazy release is tests/test_gpu_lazy_release.py
    sv = np.unique(verts).astype(np.int32)
    assert len(sv) == A
    orc = O.OracleTopology(gml)
    ips_o, _, verts_o = scenario.register_hosts(orc, H, seed=1)
    assert (verts == verts_o).all()
    rows = np.unique(np.r_[np.linspace(0, A - 1, 1024).astype(np.int64), 0, 1, A - 1])
    got = full.view(A, A, 2)[torch.from_numpy(rows).cuda()].cpu().numpy()
    yield dict(top=top, orc=orc, ips=ips_o, st=st, verts=verts, sv=sv, A=A, H=H, rows=rows, got=got, full=full)
    del full
    torch.cuda.empty_cache()


@pytest.mark.timeout(90)
def test_c4_sampled_rows_bit_exact(c4):
    """1,027 full-length rows (first, second, last and 1,024 evenly spaced) of
    the 86k x 86k slab-kernel table against the oracle's Dijkstra."""
    sv, rows, got = c4["sv"], c4["rows"], c4["got"]
    olat, orel = c4["orc"].rows_parallel(sv[rows], sv, 16)
    bad = [int(rows[i]) for i in range(len(rows))
           if not (np.array_equal(bits(got[i, :, 0]), bits(olat[i])) and np.array_equal(bits(got[i, :, 1]),
                                                                                     bits(orel[i])))]
    assert not bad, f"rows differ: {bad[:8]}"


@pytest.mark.timeout(250)
def test_c4_all_rows_bit_exact(c4):
    """Every one of the 86,603 rows of the C4 table -- latencies AND
    reliabilities (the tie-dependent half, topology.c:1578-1814) -- against the
    oracle's igraph-0.8 Dijkstra, in blocks of 2,048 rows (one D2H each), the
    oracle's rows on the job's CPU share."""
    import os
    import time

    import torch
    sv, A, full = c4["sv"], c4["A"], c4["full"]
    threads = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    t0 = time.perf_counter()
    bad = []
    blk = 2048
    for b in range(0, A, blk):
        rows = np.arange(b, min(A, b + blk))
        got = full.view(A, A, 2)[b:b + len(rows)].cpu().numpy()
        olat, orel = c4["orc"].rows_parallel(sv[rows], sv, threads)
        diff = (bits(got[:, :, 0]) != bits(olat)).any(1) | (bits(got[:, :, 1]) != bits(orel)).any(1)
        bad += [int(x) for x in rows[diff]]
        del got, olat, orel
        print(f"[c4] rows {b}..{b + len(rows)} of {A} compared ({time.perf_counter() - t0:.1f}s, {threads} threads)",
              flush=True)
    assert not bad, f"{len(bad)} rows differ, first {bad[:8]}"
    torch.cuda.empty_cache()


@pytest.mark.timeout(60)
def test_c4_frontier_latencies_all_rows(c4):
    """The frontier SSSP's latencies for all 86,603 rows of C4 against the
    heap kernel's table (an independent algorithm: Dial's buckets vs igraph's
    binary heap), in blocks of 8,192 rows compared on the device."""
    import time

    import torch
    top, A, full = c4["top"], c4["A"], c4["full"]
    blk = 8192
    d = torch.empty(blk * A, dtype=torch.float64, device="cuda")
    t0 = time.perf_counter()
    for b in range(0, A, blk):
        e = min(A, b + blk)
        top.latency_rows_frontier(b, e, d.data_ptr())
        assert torch.equal(d[:(e - b) * A].view(e - b, A), full.view(A, A, 2)[b:e, :, 0]), f"rows {b}..{e}"
        print(f"[c4] frontier rows {b}..{e} equal ({time.perf_counter() - t0:.1f}s)", flush=True)
    del d
    torch.cuda.empty_cache()


@pytest.mark.timeout(60)
def test_c4_round_all_hosts_bit_exact(c4):
    """A device-resident C4 round (1M packets) whose packets involve all 200k
    hosts: every pair's owner row (the lower slot: rows released in slot
    order) is one of the sampled rows, the other endpoint is uniform over the
    hosts of higher slots, in either direction.  The oracle holds exactly the
    sampled rows, stored in slot order as the touch order would."""
    top, orc, sv, rows, got, H = c4["top"], c4["orc"], c4["sv"], c4["rows"], c4["got"], c4["H"]
    slot_of_vertex = np.full(sv.max() + 1, -1, dtype=np.int64)
    slot_of_vertex[sv] = np.arange(len(sv))
    hslot = slot_of_vertex[c4["verts"]]
    order = np.argsort(hslot, kind="stable")
    hs_sorted = hslot[order]
    n = 1_000_000
    rng = np.random.default_rng(0x5EED0404)
    r = rows[rng.integers(0, len(rows), n)]
    owner_hosts = [order[np.searchsorted(hs_sorted, x):np.searchsorted(hs_sorted, x, "right")] for x in rows]
    pick = {x: owner_hosts[i] for i, x in enumerate(rows)}
    a = np.array([pick[x][k % len(pick[x])] for x, k in zip(r, rng.integers(0, 1 << 30, n))], dtype=np.int64)
    lo = np.searchsorted(hs_sorted, r)  # hosts with slot >= owner slot
    b = order[lo + (rng.integers(0, 1 << 62, n) % (H - lo))]
    same = a == b
    b[same] = order[np.minimum(lo[same] + 1, H - 1)]
    flip = rng.integers(0, 2, n).astype(bool)
    src, dst = np.where(flip, b, a), np.where(flip, a, b)
    keep = src != dst
    src, dst = src[keep], dst[keep]
    assert (np.minimum(hslot[src], hslot[dst])[:, None] == rows[None, :]).any(1).all()
    assert len(np.unique(dst)) > 100_000  # destinations span the host range (about 145k of 200k)
    orc.preload_rows(sv[rows], sv, got[:, :, 0], got[:, :, 1])
    pk = synth.packet_batch(len(src), H, 0x5EED0405, 100_000_000, 10_000_000, c4["st"], pairs=(src, dst))
    out, offs, status, mt = device_round(top, pk, H)
    oout, ostatus, omt = orc.round(c4["ips"], pk, BARRIER, END)
    assert np.array_equal(status, ostatus)
    assert mt == omt
    assert offs[-1] == len(out) and np.array_equal(np.diff(offs), np.bincount(oout["dst_host"], minlength=H))
    assert np.array_equal(out, oout)
    # path packet counters of the round (worker.c:551): every counter of the
    # 1,027 owner rows against the restatement, 20k pairs against the oracle
    A = c4["A"]
    keys, counts = count_check.expected_keys(hslot, pk, ostatus, A)
    assert (keys // A >= 0).all() and np.isin(keys // A, rows).all()
    count_check.check_rows(top, keys, counts, A, rows)
    k = rng.integers(0, len(pk), 20_000)
    for x, y in zip(pk["src_host"][k], pk["dst_host"][k]):
        assert top.path_packet_count(int(c4["ips"][x]), int(c4["ips"][y])) == orc.packet_count(int(c4["ips"][x]),
                                                                                                  int(c4["ips"][y]))
