"""The 8-byte packet-path table (packet.hip kPtabFallback, shd_ensure_ptab).

The rounds read {u32 delay_ns, u32 keep threshold} per entry instead of the
16-byte {lat_ms, rel}: delay_ns = (u64)ceil(lat * 1e6) (worker.c:548) and
keep_thr = max{r : (double)r / 2147483647.0 <= rel} over the 31-bit rand_r
outputs, so `chance <= rel` (worker.c:545, random.c:32-43) is `r <= keep_thr`
exactly; entries that do not fit (delay >= 2^32 - 1 ns, negative values) are
marked and decided from the f64 entry.  Checked here entry by entry against
the definition (numpy's IEEE division and ceil), at the boundaries k /
(2^31 - 1) and their neighbours, and end to end: the same rounds with and
without the table (SHD_PTAB=0) against the oracle.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_ctypes as O
from shadow_amd import _lib, scenario, synth

pytestmark = pytest.mark.gpu

M31 = 2147483647.0
FALLBACK = 0xFFFFFFFF


def build_entries(lat, rel):
    """shd_dev_ptab_build over host arrays (an internal entry point of the
    library, called here as the test's probe of the conversion)."""
    import torch
    L = _lib.lib()
    f = L.shd_dev_ptab_build
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p]
    tab = torch.from_numpy(np.stack([lat, rel], axis=1).astype(np.float64).copy()).cuda()
    out = torch.empty(len(lat) * 2, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    _lib.check(f(tab.data_ptr(), len(lat), out.data_ptr(), None))
    q = out.cpu().numpy().view(np.uint32).reshape(-1, 2)
    return q[:, 0].copy(), q[:, 1].copy()


def test_entries_match_the_definition():
    rng = np.random.default_rng(0x5EED0A01)
    k = rng.integers(0, 2**31, 4000).astype(np.float64)
    exact = k / M31  # rel values that are exactly some r / (2^31 - 1)
    rel = np.concatenate([
        rng.random(20000), exact, np.nextafter(exact, 2.0), np.nextafter(exact, -1.0),
        [0.0, 1.0, 0.5, 5e-324, 1e-300, 1.0 - 2**-53, 0.95, 0.95 * 0.98 * 0.999, -1.0, 2.0, -0.0],
    ])
    n = len(rel)
    lat = np.concatenate([rng.uniform(0.001, 400.0, n - 6), [0.0, 1e-7, 4294.967294, 4294.967296, 5000.0, -1.0]])
    delay, thr = build_entries(lat, rel)
    d = np.ceil(lat * 1000000.0)
    fits = (lat >= 0) & (d < 4294967295.0) & (rel >= 0)
    assert np.array_equal(delay == FALLBACK, ~fits)
    assert np.array_equal(delay[fits], d[fits].astype(np.uint32))
    t = thr[fits].astype(np.float64)
    r = rel[fits]
    assert np.all(t / M31 <= r), "threshold keeps a draw the reference drops"
    assert np.all((t == M31) | ((t + 1.0) / M31 > r)), "threshold drops a draw the reference keeps"


@pytest.mark.parametrize("name", ["sparse300_ns", "complete40_ns", "sparse5000_hbm", "complete25_dir"])
def test_round_with_and_without_the_table(name, monkeypatch):
    import torch

    from shadow_amd import Topology
    from test_gpu_parity import GRAPHS
    gml, H = GRAPHS[name]
    top = Topology(gml)
    ips, st, verts = scenario.register_hosts(top, H, 1)
    orc = O.OracleTopology(gml)
    ips2, _, _ = scenario.register_hosts(orc, H, 1)
    top.touch_all()
    lat, rel, sv = top.table()
    orc.preload(sv, lat, rel)
    pk = synth.packet_batch(60000, H, 0x5EED0A02, 100_000_000, 10_000_000, st)
    n = len(pk)
    d_recs = torch.from_numpy(pk.view(np.uint8)).cuda()
    res = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("SHD_PTAB", mode)
        d_out = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
        d_off = torch.empty(H + 1, dtype=torch.int32, device="cuda")
        d_status = torch.empty(n, dtype=torch.uint8, device="cuda")
        d_cnt = torch.empty(2, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        top.process_device(d_recs.data_ptr(), n, 110_000_000, 10**15, 0, d_out.data_ptr(), d_off.data_ptr(),
                           d_status.data_ptr(), d_cnt.data_ptr(), 0)
        torch.cuda.synchronize()
        cnt = d_cnt.cpu().numpy().view(np.uint64)
        res[mode] = (d_out.cpu().numpy().view(synth.DELIV_DTYPE)[:cnt[0]].copy(), d_status.cpu().numpy(), int(cnt[1]))
    oout, ostatus, omt = orc.round(ips2, pk, 110_000_000, 10**15)
    for mode, (out, status, mt) in res.items():
        assert np.array_equal(status, ostatus), mode
        assert mt == omt, mode
        assert np.array_equal(out, oout), mode
    assert (ostatus == 0).sum() > 0, "some packets must be dropped for the threshold to matter"


def test_table_refused_when_it_does_not_fit(monkeypatch):
    """The 8-B table is optional: above its budget (here SHD_PTAB_MAX_BYTES=1;
    in production half the free HBM with 8 GiB headroom, routes.c) it is not
    built and the rounds decide from the f64 entries -- same results."""
    import torch

    from shadow_amd import Topology
    from test_gpu_parity import GRAPHS
    monkeypatch.setenv("SHD_PTAB_MAX_BYTES", "1")
    gml, H = GRAPHS["sparse300_ns"]
    top = Topology(gml)
    ips, st, verts = scenario.register_hosts(top, H, 1)
    orc = O.OracleTopology(gml)
    ips2, _, _ = scenario.register_hosts(orc, H, 1)
    top.touch_all()
    lat, rel, sv = top.table()
    orc.preload(sv, lat, rel)
    pk = synth.packet_batch(30000, H, 0x5EED0A03, 100_000_000, 10_000_000, st)
    n = len(pk)
    d_recs = torch.from_numpy(pk.view(np.uint8)).cuda()
    d_out = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    d_off = torch.empty(H + 1, dtype=torch.int32, device="cuda")
    d_status = torch.empty(n, dtype=torch.uint8, device="cuda")
    d_cnt = torch.empty(2, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    top.process_device(d_recs.data_ptr(), n, 110_000_000, 10**15, 0, d_out.data_ptr(), d_off.data_ptr(),
                       d_status.data_ptr(), d_cnt.data_ptr(), 0)
    torch.cuda.synchronize()
    cnt = d_cnt.cpu().numpy().view(np.uint64)
    oout, ostatus, omt = orc.round(ips2, pk, 110_000_000, 10**15)
    assert np.array_equal(d_status.cpu().numpy(), ostatus) and int(cnt[1]) == omt
    assert np.array_equal(d_out.cpu().numpy().view(synth.DELIV_DTYPE)[:cnt[0]], oout)


def test_round_retried_without_the_table_after_oom(monkeypatch):
    """A round whose workspace does not fit beside the 8-B table
    (SHD_DEBUG_WS_OOM: the per-bucket counters' allocation fails once, after
    the old buffers were freed) drops the table and runs again from the f64
    entries (shd_ptab_release_for_retry): the same results as the oracle's,
    no stale buffer freed twice, and the next round runs clean."""
    import uuid

    import torch

    from shadow_amd import Topology
    from test_gpu_parity import GRAPHS
    gml, H = GRAPHS["sparse300_ns"]
    top = Topology(gml)
    ips, st, verts = scenario.register_hosts(top, H, 1)
    orc = O.OracleTopology(gml)
    ips2, _, _ = scenario.register_hosts(orc, H, 1)
    top.touch_all()
    lat, rel, sv = top.table()
    orc.preload(sv, lat, rel)
    pk = synth.packet_batch(30000, H, 0x5EED0A04, 100_000_000, 10_000_000, st)
    n = len(pk)
    d_recs = torch.from_numpy(pk.view(np.uint8)).cuda()
    d_out = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    d_off = torch.empty(H + 1, dtype=torch.int32, device="cuda")
    d_status = torch.empty(n, dtype=torch.uint8, device="cuda")
    d_cnt = torch.empty(2, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    oout, ostatus, omt = orc.round(ips2, pk, 110_000_000, 10**15)
    monkeypatch.setenv("SHD_DEBUG_WS_OOM", uuid.uuid4().hex[:16])
    for k in range(2):  # the retried round, then a clean one on the same workspace
        top.process_device(d_recs.data_ptr(), n, 110_000_000, 10**15, 0, d_out.data_ptr(), d_off.data_ptr(),
                           d_status.data_ptr(), d_cnt.data_ptr(), 0)
        torch.cuda.synchronize()
        if k == 0:  # (the injected failure happened: its message is the thread's last error)
            assert b"injected" in (_lib.lib().shd_last_error() or b"")
        cnt = d_cnt.cpu().numpy().view(np.uint64)
        assert np.array_equal(d_status.cpu().numpy(), ostatus) and int(cnt[1]) == omt
        assert np.array_equal(d_out.cpu().numpy().view(synth.DELIV_DTYPE)[:cnt[0]], oout)
