"""Multi-rank rounds with the ranks as threads of ONE process (Shadow runs
one process with one manager, core/manager.c:543-577): one topology and one
thread per rank, all ranks on GPU 0 here.  Transports:
  * local -- shd_transport_local_new (a thread barrier plus device-to-device
    copies), world 2 and 3;
  * rccl_all -- shd_transport_rccl_new_all: the product's own RCCL
    communicator from ncclCommInitAll (ncclGroupStart / ncclSend / ncclRecv
    on the transport's streams), world 1 on the one GPU (RCCL puts one rank
    per device; the sends and receives go to self);
  * rccl_uid -- shd_transport_rccl_new, the one-process-per-GPU form (the
    unique id handed over by torch.distributed, here a world-1 gloo group).
Each rank builds its share of the rows, the C-ABI all-gather completes every
rank's table, then each rank decides its senders' packets and the events go
to their destinations' owners -- with shd_round_process_exchange (grouped,
24-B wire records) and with shd_round_process_device + shd_round_exchange;
the records also go through shd_round_route_records on a row-sharded table.
The union over ranks must equal the oracle's single round.  A rank that
fails before the exchange makes every rank fail together (no hang)."""
import threading

import numpy as np
import pytest

import oracle_ctypes as O

pytestmark = pytest.mark.gpu

H = 300
BARRIER, END = 110_000_000, 10**15
NPK = 4000


def _gml():
    from shadow_amd import synth
    return synth.sparse_graph_gml(250, 0x5EED0801, ns_variant=True)


# owner segment sizes at the grouping and merge thresholds (hot = -1)
XEDGES = [16, 17, 63, 64, 65, 127, 128, 129, 255, 256, 257, 511, 512, 513, 1023, 1024, 1025]


def _packets(rank, world, st, hot=0):
    """hot > 0: every packet goes to one of `hot` destinations spread over
    the hosts (long destination segments on the sender and the owner);
    hot = -1: destinations 2, 5, 8, ... receive XEDGES[i] events in all,
    split over the ranks, the rest of each rank's packets go elsewhere."""
    from shadow_amd import synth
    lo, hi = rank * H // world, (rank + 1) * H // world
    if hot < 0:
        rng = np.random.default_rng(0x5EED0830 + rank)
        edge_hosts = [2 + 3 * i for i in range(len(XEDGES))]
        d = np.concatenate([np.full(c // world + (1 if rank < c % world else 0), h, dtype=np.int64)
                            for h, c in zip(edge_hosts, XEDGES)])
        others = np.setdiff1d(np.arange(H), edge_hosts)
        dst = np.concatenate([d, rng.choice(others, NPK - len(d))])[rng.permutation(NPK)]
        src = rng.integers(lo, hi, NPK)
        src = np.where(src == dst, lo + (src - lo + 1) % (hi - lo), src)
        return synth.packet_batch(NPK, H, 0x5EED0810 + rank, 100_000_000, 10_000_000, st, p_payload=0.0,
                                  pairs=(src.astype(np.uint32), dst.astype(np.uint32)))
    if not hot:
        return synth.packet_batch(NPK, H, 0x5EED0810 + rank, 100_000_000, 10_000_000, st, hosts_lo=lo, hosts_hi=hi)
    rng = np.random.default_rng(0x5EED0820 + rank)
    hosts = np.array([i * H // hot for i in range(hot)] + [H // 2 + 1])
    src = rng.integers(lo, hi, NPK).astype(np.uint32)
    k = rng.integers(0, hot, NPK)
    dst = hosts[k]
    dst = np.where(dst == src, hosts[(k + 1) % len(hosts)], dst).astype(np.uint32)
    return synth.packet_batch(NPK, H, 0x5EED0810 + rank, 100_000_000, 10_000_000, st, pairs=(src, dst))


class _UidTransport:
    """shd_transport_rccl_new over a world-1 torch.distributed group."""

    def __init__(self):
        import datetime

        import torch.distributed as dist

        from shadow_amd.transport import RcclTransport
        # an in-process store: no port to race for (world 1, this process only)
        dist.init_process_group("gloo", store=dist.HashStore(), rank=0, world_size=1,
                                timeout=datetime.timedelta(seconds=60))
        self.x = RcclTransport(0)
        self.ranks = [self.x]

    def close(self):
        import torch.distributed as dist
        self.x.close()
        dist.destroy_process_group()


def _transports(kind, world):
    from shadow_amd.transport import InProcessTransports
    if kind == "local":
        return InProcessTransports(world, "local")
    if kind == "rccl_all":
        return InProcessTransports(world, "rccl", devices=[0] * world)
    return _UidTransport()


def _run_ranks(world, fn):
    errs = [None] * world
    res = [None] * world

    def main(r):
        try:
            res[r] = fn(r)
        except BaseException as e:  # reported by the main thread
            errs[r] = e

    th = [threading.Thread(target=main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in th), "a rank thread is stuck in a collective"
    return res, errs


def _setup(world, hot=0, host_bounds=None):
    import torch

    from shadow_amd import Topology, scenario
    gml = _gml()
    tops = []
    for r in range(world):
        top = Topology(gml)
        ips, st, verts = scenario.register_hosts(top, H, seed=1)
        tops.append((top, st))
    A = tops[0][0].slot_count()
    host_bounds = host_bounds or [r * H // world for r in range(world + 1)]
    bufs = []
    for r in range(world):
        cap = NPK * world
        bufs.append(dict(
            tab=torch.zeros(A * A * 2, dtype=torch.float64, device="cuda"),
            recs=torch.from_numpy(_packets(r, world, tops[r][1], hot).view(np.uint8)).cuda(),
            send=torch.empty(cap * 32, dtype=torch.uint8, device="cuda"),
            routed=torch.empty(cap * 32, dtype=torch.uint8, device="cuda"),
            off=torch.empty(H + 1, dtype=torch.int32, device="cuda"),
            status=torch.empty(cap, dtype=torch.uint8, device="cuda"),
            cnt=torch.empty(2, dtype=torch.int64, device="cuda"),
            recv=torch.empty(cap * 32, dtype=torch.uint8, device="cuda"),
            fin=torch.empty(cap * 32, dtype=torch.uint8, device="cuda"),
            fin_off=torch.empty(host_bounds[r + 1] - host_bounds[r] + 1, dtype=torch.int32, device="cuda")))
    torch.cuda.synchronize()
    return gml, tops, A, host_bounds, bufs


def _oracle_round(gml, world, hot=0):
    orc = O.OracleTopology(gml)
    from shadow_amd import scenario
    ips, st, verts = scenario.register_hosts(orc, H, 1)
    sv = np.unique(verts).astype(np.int32)
    lat, rel = orc.rows_parallel(sv, sv, 8)
    want_tab = np.stack([lat, rel], axis=-1).tobytes()
    orc.preload(sv, lat, rel)
    allpk = np.concatenate([_packets(r, world, st, hot) for r in range(world)])
    ref, status, mt = orc.round(ips, allpk, BARRIER, END)
    _oracle_round.last = (orc, ips, verts)
    return want_tab, ref, mt


def _check_counts(tops):
    """The path packet counters summed over the ranks (each counts the
    packets it decided, worker.c:551) against the oracle's single round, for
    every host pair."""
    from count_check import check_against_oracle, slot_map
    orc, ips, verts = _oracle_round.last
    C = sum(top.path_packet_counts() for top, _ in tops)
    a, b = np.meshgrid(np.arange(H), np.arange(H), indexing="ij")
    check_against_oracle(C, slot_map(verts), orc, ips, a.ravel(), b.ravel())


def _check_union(bufs, res, world, host_bounds, ref, mt, nrec=None):
    from shadow_amd import synth
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


@pytest.mark.timeout(60)
@pytest.mark.parametrize("kind,world", [("local", 2), ("local", 3), ("rccl_all", 1), ("rccl_uid", 1)])
@pytest.mark.parametrize("fused", [True, False], ids=["process_exchange", "device+exchange"])
@pytest.mark.parametrize("split", ["1", "0"], ids=["split", "one_group"])
def test_threads_as_ranks(kind, world, fused, split, monkeypatch):
    """split: shd_round_process_exchange sends in two groups (owners below W/2
    while the sender sorts the rest, then the others) -- or in one after the
    whole round (SHD_XCHG_SPLIT=0)."""
    monkeypatch.setenv("SHD_XCHG_SPLIT", split)
    gml, tops, A, host_bounds, bufs = _setup(world)
    row_bounds = [r * A // world for r in range(world + 1)]
    xps = _transports(kind, world)

    def rank_main(r):
        top, _ = tops[r]
        b, xp = bufs[r], xps.ranks[r]
        lo, hi = row_bounds[r], row_bounds[r + 1]
        if hi > lo:
            top.build_rows_device(lo, hi, b["tab"].data_ptr())
        top.allgather_rows(xp, b["tab"].data_ptr(), row_bounds)
        top.adopt_table_device(b["tab"].data_ptr())
        top.touch_all()
        if fused:
            n = top.process_exchange(xp, b["recs"].data_ptr(), NPK, BARRIER, END, 0, host_bounds,
                                     b["send"].data_ptr(), b["status"].data_ptr(), b["cnt"].data_ptr(),
                                     b["recv"].data_ptr(), NPK * world, b["fin"].data_ptr(), b["fin_off"].data_ptr())
            # this thread's phase times: a split call leaves them, one group does not
            import ctypes as C

            from shadow_amd import _lib
            ph, ok = (C.c_double * 8)(), C.c_int()
            _lib.check(_lib.lib().shd_round_exchange_phases(ph, 8, C.byref(ok)))
            split_ran = split == "1" and world >= 2 and kind == "local"
            assert ok.value == (1 if split_ran else 0)
            if split_ran:  # decide, counts, group 1, group 2, merge, call, overlap
                assert all(v >= 0 for v in ph) and ph[5] >= ph[0] and ph[5] >= ph[4], list(ph)
            return n
        top.process_device(b["recs"].data_ptr(), NPK, BARRIER, END, 0, b["send"].data_ptr(), b["off"].data_ptr(),
                           b["status"].data_ptr(), b["cnt"].data_ptr(), 0)
        return top.exchange(xp, b["send"].data_ptr(), b["off"].data_ptr(), host_bounds, b["recv"].data_ptr(),
                            NPK * world, b["fin"].data_ptr(), b["fin_off"].data_ptr())

    try:
        res, errs = _run_ranks(world, rank_main)
        assert not any(errs), [e for e in errs if e]
    finally:
        xps.close()
    want_tab, ref, mt = _oracle_round(gml, world)
    for b in bufs:  # every rank's all-gathered table
        assert b["tab"].cpu().numpy().tobytes() == want_tab
    _check_union(bufs, res, world, host_bounds, ref, mt)
    _check_counts(tops)


@pytest.mark.timeout(60)
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("hot", [1, 2, 6, -1], ids=["hot1", "hot2", "hot6", "edges"])
@pytest.mark.parametrize("wire_sorted", ["1", "0"], ids=["sorted_wire", "unsorted_wire"])
@pytest.mark.parametrize("split", ["1", "0"], ids=["split", "one_group"])
def test_exchange_long_segments(world, hot, wire_sorted, split, monkeypatch):
    """Packets aimed at a few hot destinations: sender segments past the
    part sort's LDS capacity (listed, sorted, converted to wire records) and
    owner segments past the run merge's LDS stage (kMergeMax: listed) or
    below it (merged from sorted runs of hundreds); SHD_WIRE_SORTED=0 sends
    unsorted runs that the owner sorts."""
    monkeypatch.setenv("SHD_WIRE_SORTED", wire_sorted)
    monkeypatch.setenv("SHD_XCHG_SPLIT", split)
    gml, tops, A, host_bounds, bufs = _setup(world, hot)
    xps = _transports("local", world)

    def rank_main(r):
        top, _ = tops[r]
        b, xp = bufs[r], xps.ranks[r]
        top.build_rows_device(0, A, b["tab"].data_ptr())
        top.adopt_table_device(b["tab"].data_ptr())
        top.touch_all()
        return top.process_exchange(xp, b["recs"].data_ptr(), NPK, BARRIER, END, 0, host_bounds,
                                    b["send"].data_ptr(), b["status"].data_ptr(), b["cnt"].data_ptr(),
                                    b["recv"].data_ptr(), NPK * world, b["fin"].data_ptr(), b["fin_off"].data_ptr())

    try:
        res, errs = _run_ranks(world, rank_main)
        assert not any(errs), [e for e in errs if e]
    finally:
        xps.close()
    _, ref, mt = _oracle_round(gml, world, hot)
    _check_union(bufs, res, world, host_bounds, ref, mt)
    _check_counts(tops)


@pytest.mark.timeout(60)
@pytest.mark.parametrize("bounds", [[0, 1, 64, 200, H], [0, 150, 150, 151, H], [0, 0, 0, 0, H], [0, H, H, H, H],
                                    [0, 37, 38, 299, H]], ids=["ragged", "empty_mid", "last_owns_all",
                                                               "first_owns_all", "singletons"])
@pytest.mark.parametrize("split", ["1", "0"], ids=["split", "one_group"])
def test_uneven_owner_bounds(bounds, split, monkeypatch):
    """Owner ranges of every shape on 4 ranks: single hosts, empty ranges,
    one rank owning every destination.  The split exchange cuts each
    sender's sorted events at these bounds before the sort (k_part_cuts) and
    sends owners below W/2 first; the union must still equal the oracle."""
    monkeypatch.setenv("SHD_XCHG_SPLIT", split)
    world = 4
    gml, tops, A, host_bounds, bufs = _setup(world, host_bounds=bounds)
    xps = _transports("local", world)

    def rank_main(r):
        top, _ = tops[r]
        b, xp = bufs[r], xps.ranks[r]
        top.build_rows_device(0, A, b["tab"].data_ptr())
        top.adopt_table_device(b["tab"].data_ptr())
        top.touch_all()
        return top.process_exchange(xp, b["recs"].data_ptr(), NPK, BARRIER, END, 0, host_bounds,
                                    b["send"].data_ptr(), b["status"].data_ptr(), b["cnt"].data_ptr(),
                                    b["recv"].data_ptr(), NPK * world, b["fin"].data_ptr(), b["fin_off"].data_ptr())

    try:
        res, errs = _run_ranks(world, rank_main)
        assert not any(errs), [e for e in errs if e]
    finally:
        xps.close()
    _, ref, mt = _oracle_round(gml, world)
    _check_union(bufs, res, world, host_bounds, ref, mt)
    _check_counts(tops)


@pytest.mark.timeout(60)
@pytest.mark.parametrize("kind,world", [("local", 2), ("rccl_all", 1)])
def test_row_sharded_route_decide_exchange(kind, world):
    """C4 at N>1: the rows stay sharded (no all-gather); every record goes to
    the rank holding its answering row (shd_round_route_records), is decided
    there on the shard, and its event to its destination's owner."""
    import torch
    gml, tops, A, host_bounds, bufs = _setup(world)
    row_bounds = [r * A // world for r in range(world + 1)]
    xps = _transports(kind, world)
    for r in range(world):  # full tables built once, then each rank adopts only its shard
        tops[r][0].build_rows_device(0, A, bufs[r]["tab"].data_ptr())
    torch.cuda.synchronize()
    shards = [bufs[r]["tab"].view(A, A * 2)[row_bounds[r]:row_bounds[r + 1]].clone() for r in range(world)]
    gmin = min(tops[r][0].shard_min_latency(shards[r].data_ptr(), row_bounds[r], row_bounds[r + 1])
               for r in range(world) if row_bounds[r + 1] > row_bounds[r])

    def rank_main(r):
        top, _ = tops[r]
        b, xp = bufs[r], xps.ranks[r]
        top.adopt_table_shard_device_resident(shards[r].data_ptr(), row_bounds[r], row_bounds[r + 1], gmin)
        n = top.route_records(xp, b["recs"].data_ptr(), NPK, row_bounds, b["routed"].data_ptr(),
                              b["send"].data_ptr(), NPK * world)
        return top.process_exchange(xp, b["send"].data_ptr(), n, BARRIER, END, 0, host_bounds, b["recv"].data_ptr(),
                                    b["status"].data_ptr(), b["cnt"].data_ptr(), b["routed"].data_ptr(),
                                    NPK * world, b["fin"].data_ptr(), b["fin_off"].data_ptr())

    try:
        res, errs = _run_ranks(world, rank_main)
        assert not any(errs), [e for e in errs if e]
    finally:
        xps.close()
    _, ref, mt = _oracle_round(gml, world)
    _check_union(bufs, res, world, host_bounds, ref, mt)
    _check_counts(tops)  # (each record counted on the rank holding its answering row)


@pytest.mark.timeout(60)
@pytest.mark.parametrize("kind,world", [("local", 2), ("local", 3)])
@pytest.mark.parametrize("split", ["1", "0"], ids=["split", "one_group"])
def test_one_rank_failing_fails_every_rank(kind, world, split, monkeypatch):
    """A rank whose own stage fails before the exchange (SHD_DEBUG_FAIL_RANK)
    still joins the count all-to-all: it returns its error, every peer -EIO,
    and nobody waits in the payload collective."""
    import errno

    from shadow_amd._lib import ShdError
    gml, tops, A, host_bounds, bufs = _setup(world)
    xps = _transports(kind, world)
    monkeypatch.setenv("SHD_DEBUG_FAIL_RANK", "1")
    monkeypatch.setenv("SHD_XCHG_SPLIT", split)

    def rank_main(r):
        top, _ = tops[r]
        b, xp = bufs[r], xps.ranks[r]
        top.build_rows_device(0, A, b["tab"].data_ptr())
        top.adopt_table_device(b["tab"].data_ptr())
        top.touch_all()
        return top.process_exchange(xp, b["recs"].data_ptr(), NPK, BARRIER, END, 0, host_bounds,
                                    b["send"].data_ptr(), b["status"].data_ptr(), b["cnt"].data_ptr(),
                                    b["recv"].data_ptr(), NPK * world, b["fin"].data_ptr(), b["fin_off"].data_ptr())

    try:
        res, errs = _run_ranks(world, rank_main)
    finally:
        xps.close()
    assert all(isinstance(e, ShdError) and e.code == -errno.EIO for e in errs), errs
    assert "injected" in str(errs[1]) and all("rank 1 failed" in str(errs[r]) for r in range(world) if r != 1)


@pytest.mark.timeout(60)
@pytest.mark.parametrize("world", [2, 3])
def test_rank_failing_after_its_counts_fails_every_rank(world, monkeypatch):
    """The split exchange's late failure (SHD_DEBUG_FAIL_LATE_RANK): the rank's
    count row already went out saying it was fine, so it still sends in both
    groups; the closing status all-gather then makes every rank fail
    together (-EIO), instead of the peers merging its half-written blocks
    and returning 0."""
    import errno

    from shadow_amd._lib import ShdError
    gml, tops, A, host_bounds, bufs = _setup(world)
    xps = _transports("local", world)
    monkeypatch.setenv("SHD_DEBUG_FAIL_LATE_RANK", "1")
    monkeypatch.setenv("SHD_XCHG_SPLIT", "1")

    def rank_main(r):
        top, _ = tops[r]
        b, xp = bufs[r], xps.ranks[r]
        top.build_rows_device(0, A, b["tab"].data_ptr())
        top.adopt_table_device(b["tab"].data_ptr())
        top.touch_all()
        return top.process_exchange(xp, b["recs"].data_ptr(), NPK, BARRIER, END, 0, host_bounds,
                                    b["send"].data_ptr(), b["status"].data_ptr(), b["cnt"].data_ptr(),
                                    b["recv"].data_ptr(), NPK * world, b["fin"].data_ptr(), b["fin_off"].data_ptr())

    try:
        res, errs = _run_ranks(world, rank_main)
    finally:
        xps.close()
    assert all(isinstance(e, ShdError) and e.code == -errno.EIO for e in errs), errs
    assert "injected late" in str(errs[1])
    assert all("rank 1 failed during the exchange" in str(errs[r]) for r in range(world) if r != 1), errs
