"""Lazy row release on device-resident tables.

The reference releases a source row the first time a lookup misses it
(topology.c:1900-1981 -> _topology_computeSourcePaths), stores each unordered
pair from whichever of its rows was touched first (_topology_shouldStorePath /
_topology_storePathInCache, topology.c:1189-1265) and lowers the running
minimum that feeds worker_updateMinTimeJump entry by entry (:1253-1264,
controller.c:141-153).  A device-resident table (no host mirror; C4's is
120 GB) reproduces that with a device pass over each row at its first touch
(release.hip).  These tests interleave topology_getLatency /
getReliability / isRoutable calls with worker_sendPacket-style appends
(shd_round_append_worker, two workers) in a random order on DIRECTED
ns-resolution graphs (where the owner row of a pair changes its value), and
compare, after every operation, the returned values, the running minimum and
the controller's next min-jump time with the oracle replaying the same
serial sequence on its lazy cache -- the oracle holds only the rows that
sequence touched.  The round is then collected and compared with the
oracle's round over the same records (owners decide delays and drops).

The per-entry callback order inside one row follows glib's hash iteration
order of verticesWithAttachedHosts in the reference (topology.c:1391-1409,
unspecified), so the callback *count* is not a parity target; the minimum
and the controller's next jump after every operation are.
"""
import ctypes as C
import time

import numpy as np
import pytest

import oracle_ctypes as O
from shadow_amd import Topology, _lib, scenario, synth

pytestmark = pytest.mark.gpu

BARRIER, END = 110_000_000, 10**15


def bits(x):
    return np.float64(x).view(np.uint64)


T0 = [time.perf_counter()]


def progress(*a):
    """Progress lines (pytest -s): the long cases must not look hung."""
    print(f"[lazy {time.perf_counter() - T0[0]:7.1f}s]", *a, flush=True)


def interleave_check(top, orc, ips, st, H, pool, n_lookups, n_sends, seed, workers=2, check_log=False,
                     check_every=1):
    """Random interleaving of lookups and send chunks over the host `pool`;
    returns the number of rows the sequence touched (product view)."""
    lib = _lib.lib()
    rng = np.random.default_rng(seed)
    kinds = rng.permutation(np.r_[np.zeros(n_lookups, np.int64), np.ones(n_sends, np.int64)])
    a = pool[rng.integers(0, len(pool), len(kinds))]
    b = pool[rng.integers(0, len(pool), len(kinds))]
    sends = np.flatnonzero(kinds == 1)
    same = a[sends] == b[sends]
    b[sends[same]] = pool[(np.searchsorted(pool, a[sends[same]]) + 1) % len(pool)]
    pk = synth.packet_batch(len(sends), H, seed & 0xFFFFFFFF, 100_000_000, 10_000_000, st,
                            pairs=(a[sends], b[sends]))
    top.record_min_jump()
    _lib.check(lib.shd_round_set_workers(top.handle, workers))
    _lib.check(lib.shd_round_begin(top.handle, BARRIER, END, 0))
    per_worker = [[] for _ in range(workers)]
    i, j, chunk, step = 0, 0, 0, 0
    lk = rng.integers(0, 3, len(kinds))
    while i < len(kinds):
        if kinds[i] == 0:
            s, d = int(ips[a[i]]), int(ips[b[i]])
            if lk[i] == 0:
                assert bits(top.get_latency(s, d)) == bits(orc.latency(s, d)), (i, a[i], b[i])
            elif lk[i] == 1:
                assert bits(top.get_reliability(s, d)) == bits(orc.reliability(s, d)), (i, a[i], b[i])
            else:
                assert top.is_routable(s, d) == orc.routable(s, d)
            i += 1
        else:
            k = i
            while k < len(kinds) and kinds[k] == 1 and k - i < 64:
                k += 1
            recs = np.ascontiguousarray(pk[j:j + (k - i)])
            w = chunk % workers
            _lib.check(lib.shd_round_append_worker(top.handle, w, recs.ctypes.data, len(recs)))
            for r in recs:  # worker_sendPacket's lookup (worker.c:539), in send order
                orc.reliability(int(ips[r["src_host"]]), int(ips[r["dst_host"]]))
            per_worker[w].append(recs)
            j += k - i
            i = k
            chunk += 1
        step += 1
        if step % 500 == 0:
            progress(f"op {i}/{len(kinds)}")
        if step % check_every == 0 or i == len(kinds):
            assert bits(top.min_path_latency()) == bits(orc.min_path_latency()), (i, step)
            assert top.next_min_jump_ns() == orc.next_min_jump_ns(), (i, step)
    staged = np.concatenate([np.concatenate(x) if x else pk[:0] for x in per_worker])  # worker order
    n = len(staged)
    out = np.zeros(max(n, 1), dtype=synth.DELIV_DTYPE)
    offs = np.zeros(H + 1, dtype=np.uint32)
    status = np.zeros(max(n, 1), dtype=np.uint8)
    nout, mt = C.c_size_t(), C.c_uint64()
    _lib.check(lib.shd_round_collect(top.handle, out.ctypes.data, len(out), C.byref(nout), offs.ctypes.data,
                                     status.ctypes.data, C.byref(mt)))
    progress(f"collected {nout.value} events of {n} records")
    oout, ostatus, omt = orc.round(ips, staged, BARRIER, END)  # every lookup is a hit now
    progress("oracle round done")
    assert np.array_equal(status[:n], ostatus)
    assert mt.value == omt
    assert np.array_equal(out[:nout.value], oout)
    assert np.array_equal(np.diff(offs.astype(np.int64)), np.bincount(oout["dst_host"], minlength=H))
    assert top.min_jump_calls == sorted(set(top.min_jump_calls), reverse=True)  # strictly decreasing
    if check_log:
        assert top.cached_paths_log() == orc.cached_paths_log()
    seq = np.empty(top.slot_count(), dtype=np.uint32)
    _lib.check(lib.shd_topology_touch_order(top.handle, seq.ctypes.data, None, len(seq)))
    progress("compared")
    return int((seq != 0xFFFFFFFF).sum())


def setup(gml, H, shards):
    """Product topology with a device-resident table (one shard, or `shards`
    shards of a single-process multi-GPU table, all on GPU 0 here) + oracle."""
    import torch
    progress(f"setup H={H} shards={shards}")
    top = Topology(gml)
    ips, st, verts = scenario.register_hosts(top, H, seed=1)
    orc = O.OracleTopology(gml)
    _, st2, verts2 = scenario.register_hosts(orc, H, seed=1)
    assert (verts == verts2).all() and (st == st2).all()
    A = top.slot_count()
    bounds = [A * k // shards for k in range(shards + 1)]
    bufs = [torch.empty(max(bounds[k + 1] - bounds[k], 1) * A * 2, dtype=torch.float64, device="cuda")
            for k in range(shards)]
    if shards == 1:
        top.build_rows_device(0, A, bufs[0].data_ptr())
        torch.cuda.synchronize()
        top.adopt_table_device_resident(bufs[0].data_ptr())
    else:
        top.build_shards([0] * shards, [b.data_ptr() for b in bufs], bounds)
        torch.cuda.synchronize()
        top.adopt_table_shards([0] * shards, [b.data_ptr() for b in bufs], bounds)
    progress(f"table A={A} built and adopted")
    assert top.min_path_latency() == 0  # nothing released at adoption
    return top, orc, ips, st, bufs


@pytest.mark.timeout(60)
@pytest.mark.parametrize("shards", [1, 2, 3])
@pytest.mark.parametrize("name", ["sparse3000_dir_ns", "sparse5000_dir_ns_hbm"])
def test_lazy_release_small(name, shards):
    """Every host of a 3,000 / 5,000-vertex directed ns graph in play, so most
    rows get touched in a random order; the teardown log (which pairs are
    stored, from which row) must equal the oracle's cache line for line."""
    V = {"sparse3000_dir_ns": 3000, "sparse5000_dir_ns_hbm": 5000}[name]
    gml = synth.sparse_graph_gml(V, 0x5EED0900 + V, ns_variant=True, directed=True)
    H = 2 * V
    top, orc, ips, st, bufs = setup(gml, H, shards)
    pool = np.arange(H)
    touched = interleave_check(top, orc, ips, st, H, pool, 3000, 6000, 0x5EED0910 + V + shards, check_log=True)
    assert touched > 1000


@pytest.mark.timeout(60)
def test_lazy_release_c2_two_shards():
    """configs[2]'s size -- V = 20k, H = 50k -- as a directed ns graph on a
    single-process two-shard table (Shadow's one process, core/manager.c:
    543-577, with its rows split over two devices; both on GPU 0 here): one
    release state, row passes on the owning shard, the round decided on the
    shard of each record's answering row and regrouped at the destination's
    shard."""
    gml = synth.sparse_graph_gml(20_000, 0x5EED0920, ns_variant=True, directed=True)
    H = 50_000
    top, orc, ips, st, bufs = setup(gml, H, 2)
    pool = np.unique(np.random.default_rng(7).integers(0, H, 600))
    touched = interleave_check(top, orc, ips, st, H, pool, 2000, 20000, 0x5EED0921, check_every=8)
    assert touched > 300


@pytest.mark.timeout(60)
def test_lazy_release_c4_device_resident():
    """configs[4]'s size -- V = 100k, H = 200k, the 120 GB table with no host
    mirror -- as a directed ns graph: lookups and sends among 240 hosts in a
    random order; the oracle computes only the rows the sequence touches."""
    import torch
    T0[0] = time.perf_counter()
    gml = synth.sparse_graph_gml(100_000, 0x5EED0930, ns_variant=True, directed=True)
    H = 200_000
    top, orc, ips, st, bufs = setup(gml, H, 1)
    pool = np.unique(np.random.default_rng(8).integers(0, H, 240))
    touched = interleave_check(top, orc, ips, st, H, pool, 1500, 8000, 0x5EED0931, check_every=16)
    assert touched > 150
    top.close()  # before the table it reads goes away
    orc.close()
    progress("closed")
    del bufs
    torch.cuda.empty_cache()
    progress("table freed")
