"""GPU parity for the destination routers (shd_codel_run):
libshdnet's one-lane-per-router CoDel engine against the oracle's
restatement of routing/router_queue_codel.c:113-265, bit-exact in every
output: per-op packet, per-packet fate (op index + status), every state
field (f64 control law included) and the entries left queued."""
import numpy as np
import pytest

import oracle_ctypes as O
from shadow_amd import ShdError, Topology, scenario, synth
from shadow_amd.router import DEQUEUE, DROPPED, ENQUEUE, OP_DTYPE, CodelRouters, trace_from_arrivals

pytestmark = pytest.mark.gpu
MS = 1_000_000


def _compare(G, R, deq_g, fate_g, deq_o, fate_o):
    assert np.array_equal(deq_g, deq_o)
    assert np.array_equal(fate_g, fate_o)
    sg = G.state()
    for k in sg.dtype.names:
        assert np.array_equal(sg[k], R.states[k]), k
    ring = G.rings.cpu().numpy().view(R.rings.dtype).reshape(G.n, G.cap)
    live = (sg["head"][:, None] + np.arange(G.cap)[None, :]) % G.cap
    mask = np.arange(G.cap)[None, :] < sg["len"][:, None]
    got = np.take_along_axis(ring, live, axis=1)[mask]
    want = np.take_along_axis(R.rings.reshape(G.n, G.cap), live, axis=1)[mask]
    assert np.array_equal(got, want)


def _random(nr, seed, npr, span=400 * MS):
    rng = np.random.default_rng(seed)
    router = np.sort(rng.integers(0, nr, nr * npr))
    arr = np.sort(rng.integers(0, span, len(router)))
    arr = arr[np.argsort(router, kind="stable")]  # per router non-decreasing
    return router, arr, rng.integers(60, 1500, len(router))


def test_known_answer_on_gpu():
    rows = [(0, ENQUEUE, k) for k in range(10)] + [(20 * MS, DEQUEUE, 0), (130 * MS, DEQUEUE, 0),
                                                  (240 * MS, DEQUEUE, 0)]
    ops = np.zeros(len(rows), dtype=OP_DTYPE)
    for i, (t, kind, p) in enumerate(rows):
        ops[i] = (t, kind, p, 1500, 0)
    off = np.array([0, len(rows)], np.uint32)
    G, R = CodelRouters(1, 16), O.OracleRouters(1, 16)
    deq_g, fate_g = G.run(off, ops, 10)
    rc, deq_o, fate_o = R.run(off, ops, 10)
    assert rc == 0 and list(deq_g[10:]) == [0, 2, 9]
    _compare(G, R, deq_g, fate_g, deq_o, fate_o)


@pytest.mark.parametrize("svc", [20.0, 8_000.0, 40_000.0])
def test_random_traces_bit_exact(svc):
    """20k routers, ~30 packets each: idle (20 ns/B), near capacity and
    heavily overloaded (drop mode and the control law's drop loop)."""
    nr = 20_000
    router, arr, length = _random(nr, 0x5EED0C00 + int(svc), 30)
    off, ops = trace_from_arrivals(router, arr, length, nr, svc)
    G, R = CodelRouters(nr, 256), O.OracleRouters(nr, 256)
    deq_g, fate_g = G.run(off, ops, len(router))
    rc, deq_o, fate_o = R.run(off, ops, len(router))
    assert rc == 0
    _compare(G, R, deq_g, fate_g, deq_o, fate_o)
    if svc > 1000:
        assert ((fate_g & np.uint64(3)) == DROPPED).sum() > 0


def test_batches_carry_state_on_device():
    """Three batches (a third of each router's ops each), state and queued
    entries resident on the device between them, against the oracle fed the
    same batches."""
    nr = 5000
    router, arr, length = _random(nr, 0x5EED0C10, 40)
    off, ops = trace_from_arrivals(router, arr, length, nr, 15_000.0)
    G, R = CodelRouters(nr, 512), O.OracleRouters(nr, 512)
    cuts = [off[:-1] + (off[1:] - off[:-1]) * k // 3 for k in range(4)]
    carried = False
    for b in range(3):
        idx = np.concatenate([np.arange(cuts[b][r], cuts[b + 1][r]) for r in range(nr)]).astype(np.int64)
        o = np.r_[0, np.cumsum(cuts[b + 1].astype(np.int64) - cuts[b])].astype(np.uint32)
        deq_g, fate_g = G.run(o, ops[idx], len(router))
        rc, deq_o, fate_o = R.run(o, ops[idx], len(router))
        assert rc == 0
        _compare(G, R, deq_g, fate_g, deq_o, fate_o)
        if b < 2:  # packets queued at a batch boundary carry over (the trace drains by its end)
            carried |= bool((G.state()["len"] > 0).any())
    assert carried


def test_errors_fail_loudly():
    G = CodelRouters(2, 2)
    ops = np.zeros(4, dtype=OP_DTYPE)
    ops["kind"] = [DEQUEUE, ENQUEUE, ENQUEUE, ENQUEUE]
    ops["pkt"] = [0, 0, 1, 2]
    ops["time"] = [5, 0, 1, 2]
    ops["length"] = 1500
    with pytest.raises(ShdError) as e:
        G.run(np.array([0, 1, 4], np.uint32), ops, 3)
    assert e.value.code == -28  # -ENOSPC
    G2 = CodelRouters(1, 4)
    ops2 = np.zeros(2, dtype=OP_DTYPE)
    ops2["kind"], ops2["time"], ops2["length"] = [ENQUEUE, DEQUEUE], [10, 5], 1500
    with pytest.raises(ShdError) as e:
        G2.run(np.array([0, 2], np.uint32), ops2, 1)
    assert e.value.code == -22  # -EINVAL


def test_routers_fed_by_a_round():
    """The delivered events of a hand-off round, per destination in
    event_compare order, become each destination router's arrivals."""
    gml = synth.sparse_graph_gml(300, 0x5EED0C20)
    H = 400
    top = Topology(gml)
    ips, st, verts = scenario.register_hosts(top, H, 1)
    pk = synth.packet_batch(60_000, H, 0x5EED0C21, 100_000_000, 10_000_000, st, zipf=True)
    out, offs, status, mt = top.round(pk, 110_000_000, 10**15)
    length = pk["payload_len"][out["pkt_index"]].astype(np.int64) + 52
    off, ops = trace_from_arrivals(out["dst_host"], out["time"], length, H, 400.0)
    cap = int(np.bincount(out["dst_host"], minlength=H).max()) + 1
    G, R = CodelRouters(H, cap), O.OracleRouters(H, cap)
    deq_g, fate_g = G.run(off, ops, len(out))
    rc, deq_o, fate_o = R.run(off, ops, len(out))
    assert rc == 0
    _compare(G, R, deq_g, fate_g, deq_o, fate_o)
