"""Network interfaces (token buckets + refill grid + upstream CoDel router)
on the CPU oracle: hand-derived known answers from host/network_interface.c
and routing/router.c, and window splitting.  The reference ships no
interface test or fixture: the known answers below pin this row (worked by
hand from the code), otherwise "parity unpinned"."""
import numpy as np

import oracle_ctypes as O
from shadow_amd.router import NIC_DROPPED, NIC_QUEUED, NIC_RECEIVED, SEND_DTYPE
from shadow_amd.synth import DELIV_DTYPE

MS = 1_000_000
NEVER = np.uint64(0xFFFFFFFFFFFFFFFF)


def _events(rows, dst):
    ev = np.zeros(len(rows), dtype=DELIV_DTYPE)
    for i, (t, src) in enumerate(rows):
        ev[i] = (t, i, src, dst, i, 0)
    return ev


def test_receive_bucket_known_answer():
    """2930 KiB/s down -> 3000 B per 1 ms refill, capacity 4500.  Four
    1500-byte packets from host 0 at 0.1-0.4 ms: the first two are pulled at
    once (3000 B), the next two wait in the router for the 1 ms refill."""
    nic = O.OracleInterfaces(1, [2930], [10**6], 0, 16, 4, host_base=1)
    st = nic.states[0]
    assert (int(st["recv_refill"]), int(st["recv_capacity"]), int(st["recv_remaining"])) == (3000, 4500, 3000)
    assert int(st["refill_pending"]) == 1 and int(st["refill_time"]) == MS
    ev = _events([(MS // 10 * k, 0) for k in (1, 2, 3, 4)], 1)
    nic.run(ev, [0, 4], [1500] * 4, 3 * MS)
    assert nic.recv_time.tolist() == [MS // 10, 2 * MS // 10, MS, MS]
    assert (nic.recv_status == NIC_RECEIVED).all()
    st = nic.states[0]
    assert int(st["recv_remaining"]) == 3000 and int(st["refill_time"]) == 3 * MS and int(st["refill_pending"]) == 1


def test_send_bucket_known_answer_and_bootstrap():
    """2930 KiB/s up: five 1000-byte packets offered at 0.1 ms: two leave at
    once (3000 -> 1000 B left < MTU), three at the 1 ms refill.  While
    bootstrapping nothing is consumed and all five leave at 0.1 ms."""
    sends = np.zeros(5, dtype=SEND_DTYPE)
    sends["ready"], sends["id"], sends["length"] = MS // 10, np.arange(5), 1000
    ev = np.zeros(0, dtype=DELIV_DTYPE)
    nic = O.OracleInterfaces(1, [10**6], [2930], 0, 4, 1)
    t = nic.run(ev, [0, 0], [], 2 * MS, sends=sends, send_offsets=[0, 5])
    assert t.tolist() == [MS // 10] * 2 + [MS] * 3
    nic = O.OracleInterfaces(1, [10**6], [2930], 0, 4, 1)
    t = nic.run(ev, [0, 0], [], 2 * MS, bootstrap_end=MS // 2, sends=sends, send_offsets=[0, 5])
    assert t.tolist() == [MS // 10] * 5


def test_router_drops_under_a_slow_receiver():
    """A 100 KiB/s receiver (102 B per ms) fed 1500-byte packets every ms for
    a second: the router's standing queue exceeds CoDel's target and some
    packets are dropped (PDS_ROUTER_DROPPED)."""
    n = 1000
    nic = O.OracleInterfaces(1, [100], [10**6], 0, 4096, n, host_base=3)
    ev = _events([(k * MS + 17, 0) for k in range(n)], 3)
    nic.run(ev, [0, n], [1500] * n, (n + 5) * MS)
    st = nic.recv_status
    assert (st == NIC_DROPPED).sum() > 0 and (st == NIC_RECEIVED).sum() > 0
    assert (st == NIC_QUEUED).sum() == int(nic.states[0]["router"]["len"])


def _random_case(nh, seed, per=300, span=300 * MS):
    rng = np.random.default_rng(seed)
    rows = []
    for h in range(nh):
        k = int(rng.integers(0, per))
        t = np.sort(rng.integers(0, span, k) // (MS // 2) * (MS // 2) + rng.integers(0, 2, k))  # many on the grid
        src = rng.integers(0, nh, k)
        src[src == h] = (h + 1) % nh
        seq = np.arange(k)
        o = np.lexsort((seq, src, t))
        for j in o:
            rows.append((int(t[j]), int(src[j]), h))
    ev = np.zeros(len(rows), dtype=DELIV_DTYPE)
    for i, (t, s, d) in enumerate(rows):
        ev[i] = (t, i, s, d, i, 0)
    off = np.zeros(nh + 1, np.uint32)
    np.cumsum(np.bincount(ev["dst_host"].astype(np.int64), minlength=nh), out=off[1:])
    lengths = rng.integers(42, 1600, len(ev)).astype(np.uint32)
    ns = rng.integers(0, per, nh)
    sends = np.zeros(int(ns.sum()), dtype=SEND_DTYPE)
    so = np.zeros(nh + 1, np.uint32)
    np.cumsum(ns, out=so[1:])
    for h in range(nh):
        sends["ready"][so[h]:so[h + 1]] = np.sort(rng.integers(0, span, ns[h]) // (MS // 2) * (MS // 2))
    sends["id"] = np.arange(len(sends))
    sends["length"] = rng.integers(42, 1600, len(sends))
    down = rng.integers(20, 3000, nh)
    up = rng.integers(20, 3000, nh)
    return ev, off, lengths, sends, so, down, up


def test_two_windows_equal_one():
    """Cutting the run at a window boundary (router entries and pending
    refills carried in the state, unsent requests offered again first)
    changes nothing."""
    nh = 40
    ev, off, ln, sends, so, down, up = _random_case(nh, 3)
    end = 400 * MS
    A = O.OracleInterfaces(nh, down, up, 0, 4096, len(ev))
    sa = A.run(ev, off, ln, end, sends=sends, send_offsets=so)
    assert (A.recv_status == NIC_DROPPED).sum() > 0
    cut = 150 * MS + MS // 2
    B = O.OracleInterfaces(nh, down, up, 0, 4096, len(ev))
    first = ev["time"] < cut
    idx1, idx2 = np.where(first)[0], np.where(~first)[0]
    o1 = np.zeros(nh + 1, np.uint32)
    np.cumsum(np.bincount(ev["dst_host"][first].astype(np.int64), minlength=nh), out=o1[1:])
    o2 = np.zeros(nh + 1, np.uint32)
    np.cumsum(np.bincount(ev["dst_host"][~first].astype(np.int64), minlength=nh), out=o2[1:])
    s_first = sends["ready"] < cut
    so1 = np.zeros(nh + 1, np.uint32)
    hs = np.repeat(np.arange(nh), np.diff(so))
    np.cumsum(np.bincount(hs[s_first], minlength=nh), out=so1[1:])
    st1 = B.run(ev[idx1], o1, ln[idx1], cut, sends=sends[s_first], send_offsets=so1)
    # second window: arrivals get their global ids (id_base 0, but events
    # renumbered: map through the fate arrays afterwards)
    unsent = np.where(s_first)[0][st1 == NEVER]
    later = np.where(~s_first)[0]
    nxt = np.concatenate([unsent, later])
    nxt = nxt[np.lexsort((np.arange(len(nxt)), hs[nxt]))]  # per host, carried first
    so2 = np.zeros(nh + 1, np.uint32)
    np.cumsum(np.bincount(hs[nxt], minlength=nh), out=so2[1:])
    B2 = B
    fate_t1, fate_s1 = B.recv_time.copy(), B.recv_status.copy()
    st2 = B2.run(ev[idx2], o2, ln[idx2], end, id_base=len(idx1), sends=sends[nxt], send_offsets=so2)
    # ids: window 1 arrival k -> id k (idx1[k]); window 2 arrival k -> id len(idx1)+k (idx2[k])
    rt = np.empty(len(ev), np.uint64)
    rs = np.empty(len(ev), np.uint8)
    rt[idx1], rs[idx1] = B.recv_time[:len(idx1)], B.recv_status[:len(idx1)]
    rt[idx2], rs[idx2] = B.recv_time[len(idx1):len(ev)], B.recv_status[len(idx1):len(ev)]
    assert np.array_equal(rs, A.recv_status) and np.array_equal(rt, A.recv_time)
    stime = np.full(len(sends), NEVER)
    stime[np.where(s_first)[0]] = st1
    stime[nxt] = st2
    assert np.array_equal(stime, sa)
    for k in ("recv_remaining", "send_remaining", "refill_time", "refill_pending"):
        assert np.array_equal(A.states[k], B.states[k]), k
    del fate_t1, fate_s1
