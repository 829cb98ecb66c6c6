"""GPU parity for the network interfaces (shd_nic_*):
libshdnet's one-lane-per-host engine (token buckets, the 1 ms refill grid,
the upstream CoDel router) against the oracle's event-driven restatement
of host/network_interface.c + routing/router.c, bit-exact: receive time and
status per packet, send time per request, every state field and the router
entries left queued."""
import numpy as np
import pytest
import torch

import oracle_ctypes as O
from shadow_amd import ShdError, Topology, scenario, synth
from shadow_amd.router import HEADER_UDP, NIC_DROPPED, SEND_DTYPE, Interfaces
from test_nic_cpu import MS, _events, _random_case

pytestmark = pytest.mark.gpu


def _compare(G, R, sg=None, so=None):
    t, s = G.fates()
    assert np.array_equal(s, R.recv_status)
    assert np.array_equal(t, R.recv_time)
    if sg is not None:
        assert np.array_equal(sg, so)
    st = G.state()
    for k in st.dtype.names:
        if k == "router":
            for kk in st["router"].dtype.names:
                assert np.array_equal(st["router"][kk], R.states["router"][kk]), kk
        else:
            assert np.array_equal(st[k], R.states[k]), k
    ring = G.rings.cpu().numpy().view(R.rings.dtype).reshape(G.n, G.cap)
    live = (st["router"]["head"][:, None] + np.arange(G.cap)[None, :]) % G.cap
    mask = np.arange(G.cap)[None, :] < st["router"]["len"][:, None]
    assert np.array_equal(np.take_along_axis(ring, live, axis=1)[mask],
                          np.take_along_axis(R.rings.reshape(G.n, G.cap), live, axis=1)[mask])


def test_known_answers_on_gpu():
    ev = _events([(MS // 10 * k, 0) for k in (1, 2, 3, 4)], 1)
    G = Interfaces(1, [2930], [10**6], 0, 16, 4, host_base=1)
    R = O.OracleInterfaces(1, [2930], [10**6], 0, 16, 4, host_base=1)
    G.run(ev, [0, 4], [1500] * 4, 3 * MS)
    R.run(ev, [0, 4], [1500] * 4, 3 * MS)
    assert G.fates()[0].tolist() == [MS // 10, 2 * MS // 10, MS, MS]
    _compare(G, R)
    sends = np.zeros(5, dtype=SEND_DTYPE)
    sends["ready"], sends["id"], sends["length"] = MS // 10, np.arange(5), 1000
    none = np.zeros(0, dtype=synth.DELIV_DTYPE)
    for boot in (0, MS // 2):
        G = Interfaces(1, [10**6], [2930], 0, 4, 1)
        R = O.OracleInterfaces(1, [10**6], [2930], 0, 4, 1)
        sg = G.run(none, [0, 0], [], 2 * MS, bootstrap_end=boot, sends=sends, send_offsets=[0, 5])
        so = R.run(none, [0, 0], [], 2 * MS, bootstrap_end=boot, sends=sends, send_offsets=[0, 5])
        _compare(G, R, sg, so)


@pytest.mark.parametrize("seed", [1, 2])
def test_random_hosts_bit_exact(seed):
    """3000 hosts, up to 300 arrivals and 300 send requests each over 300 ms,
    times often on the refill grid (ties with refills), bandwidths
    20-3000 KiB/s: drop mode, standing queues and idle refill gaps."""
    nh = 3000
    ev, off, ln, sends, so, down, up = _random_case(nh, 100 + seed)
    G = Interfaces(nh, down, up, 0, 1024, len(ev))
    R = O.OracleInterfaces(nh, down, up, 0, 1024, len(ev))
    end = 320 * MS
    sg = G.run(ev, off, ln, end, sends=sends, send_offsets=so)
    sr = R.run(ev, off, ln, end, sends=sends, send_offsets=so)
    _compare(G, R, sg, sr)
    assert (R.recv_status == NIC_DROPPED).sum() > 0 and (R.states["router"]["len"] > 0).any()


def test_windows_carry_on_device():
    """Three windows; router entries and pending refills carried on the
    device, unsent requests offered again first."""
    nh = 500
    ev, off, ln, sends, so, down, up = _random_case(nh, 9)
    G = Interfaces(nh, down, up, 0, 1024, len(ev))
    R = O.OracleInterfaces(nh, down, up, 0, 1024, len(ev))
    cuts = [0, 100 * MS + 1, 200 * MS, 320 * MS]
    hs = np.repeat(np.arange(nh), np.diff(so))
    carry = np.zeros(0, np.int64)
    base = 0
    for w in range(3):
        m = (ev["time"] >= cuts[w]) & (ev["time"] < cuts[w + 1])
        idx = np.where(m)[0]
        o = np.zeros(nh + 1, np.uint32)
        np.cumsum(np.bincount(ev["dst_host"][m].astype(np.int64), minlength=nh), out=o[1:])
        fresh = np.where((sends["ready"] >= cuts[w]) & (sends["ready"] < cuts[w + 1]))[0]
        nxt = np.concatenate([carry, fresh])
        nxt = nxt[np.lexsort((np.arange(len(nxt)), hs[nxt]))]
        s2 = np.zeros(nh + 1, np.uint32)
        np.cumsum(np.bincount(hs[nxt], minlength=nh), out=s2[1:])
        sg = G.run(ev[idx], o, ln[idx], cuts[w + 1], id_base=base, sends=sends[nxt], send_offsets=s2)
        sr = R.run(ev[idx], o, ln[idx], cuts[w + 1], id_base=base, sends=sends[nxt], send_offsets=s2)
        _compare(G, R, sg, sr)
        carry = nxt[sg == np.uint64(0xFFFFFFFFFFFFFFFF)]
        base += len(idx)


def test_interfaces_fed_by_a_round():
    """A hand-off round's per-destination segments feed the receive side in
    place (lengths from the packet records through shd_event_lengths)."""
    from shadow_amd._lib import lib
    gml = synth.sparse_graph_gml(300, 0x5EED0C30)
    H = 400
    top = Topology(gml)
    ips, st, verts = scenario.register_hosts(top, H, 1)
    pk = synth.packet_batch(80_000, H, 0x5EED0C31, 100_000_000, 10_000_000, st, zipf=True)
    out, offs, status, mt = top.round(pk, 110_000_000, 10**15)
    d_out = torch.from_numpy(out.view(np.uint8)).cuda()
    d_pk = torch.from_numpy(pk.view(np.uint8)).cuda()
    d_len = torch.empty(len(out), dtype=torch.int32, device="cuda")
    assert lib().shd_event_lengths(d_out.data_ptr(), len(out), d_pk.data_ptr(), HEADER_UDP, d_len.data_ptr(), None) == 0
    torch.cuda.synchronize()
    ln = d_len.cpu().numpy().view(np.uint32)
    assert np.array_equal(ln, pk["payload_len"][out["pkt_index"]] + HEADER_UDP)
    down = np.full(H, 10_240)  # 10 MiB/s
    up = np.full(H, 10_240)
    end = int(out["time"].max()) + 1
    G = Interfaces(H, down, up, 100_000_000, 1 << 15, len(out))
    R = O.OracleInterfaces(H, down, up, 100_000_000, 1 << 15, len(out))
    d_off = torch.from_numpy(offs.astype(np.uint32).view(np.int32)).cuda()
    G.run_device(d_out.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), end)
    torch.cuda.synchronize()
    R.run(out, offs, ln, end)
    _compare(G, R)


def test_errors_fail_loudly():
    ev = _events([(MS, 0)], 2)  # addressed to host 2, given to host 1
    G = Interfaces(1, [1000], [1000], 0, 4, 1, host_base=1)
    with pytest.raises(ShdError) as e:
        G.run(ev, [0, 1], [100], 2 * MS)
    assert e.value.code == -22
    ev = _events([(k * 10, 0) for k in range(8)], 1)
    G = Interfaces(1, [1], [1000], 0, 4, 8, host_base=1)  # 1 KiB/s: everything stays queued
    with pytest.raises(ShdError) as e:
        G.run(ev, [0, 8], [1500] * 8, MS // 2)
    assert e.value.code == -28
    # inputs every lane checks before anything runs: packet ids past the fate
    # arrays (-ERANGE) and events without their lengths (-EINVAL); no host's
    # state, fate or ring moves
    ev = _events([(k * 10, 0) for k in range(4)], 1)
    G = Interfaces(1, [1000], [1000], 0, 4, 4, host_base=1)
    st0, t0 = G.state().copy(), G.fates()[0].copy()
    with pytest.raises(ShdError) as e:
        G.run(ev, [0, 4], [100] * 4, MS, id_base=1)
    assert e.value.code == -34
    d_ev = torch.from_numpy(ev.view(np.uint8)).cuda()
    d_off = torch.from_numpy(np.array([0, 4], np.uint32).view(np.int32)).cuda()
    with pytest.raises(ShdError) as e:
        G.run_device(d_ev.data_ptr(), d_off.data_ptr(), 0, MS)
    assert e.value.code == -22 and "lengths" in str(e.value)
    assert G.state().tobytes() == st0.tobytes() and np.array_equal(G.fates()[0], t0)
