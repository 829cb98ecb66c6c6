"""srcHostEventID of dropped sends.

The reference takes host_getNewEventID only for a KEPT packet, inside
event_new_ (core/worker.c:565-569 -> core/work/event.c:37); the drop-in
worker_sendPacket (integration/worker_send_shdnet.c:42) reserves it at send
time for EVERY send, because the drop is decided at the round boundary.  So
after a host's first dropped packet its later ids are larger than the
reference's.  They stay strictly increasing in creation order, and
event_compare (event.c:109-152) compares srcHostEventIDs only between events
of the same (time, dst, src) -- i.e. of one sender -- so the delivered order
is the same.  This test replays one round on the oracle twice: with the
reference's ids (only kept packets, plus interleaved non-packet events, take
ids) and with the drop-in's (every send takes one), on a batch built so that
(time, dst, src) ties are frequent (the id decides them) and with self-sends.
The orders must be identical, the absolute ids must differ.
"""
import numpy as np

import oracle_ctypes as O
from shadow_amd import scenario, synth

KEPT = (1, 2)  # delivered, dropped at the end time: both created their event (worker.c:565)


def test_dropped_sends_consume_ids_order_unchanged():
    gml = synth.complete_graph_gml(12, 0x5EED0E01)
    H, n = 24, 6000
    rng = np.random.default_rng(0x5EED0E02)
    src = rng.integers(0, H, n).astype(np.uint32)
    dst = np.where(rng.random(n) < 0.15, src, rng.integers(0, 4, n)).astype(np.uint32)  # few dsts + self-sends
    orc = O.OracleTopology(gml)
    ips, st, _ = scenario.register_hosts(orc, H, seed=1)
    pk = synth.packet_batch(n, H, 0x5EED0E03, 100_000_000, 10_000_000, st, pairs=(src, dst))
    pk["now"] = 100_000_000 + (pk["now"] - 100_000_000) // 2_000_000 * 2_000_000  # coarse times: (time, dst, src) ties
    pk["payload_len"] = 1448
    # decide once to learn which sends are kept (the draw does not depend on the id)
    _, status, _ = orc.round(ips, pk, 110_000_000, 150_000_000)
    kept = np.isin(status, KEPT)
    assert 0 < (~kept).sum() < n and (status == 2).sum() > 0
    # per sender, in send order: the drop-in's id = every send, the
    # reference's = kept sends only; both interleaved with the host's other
    # events (gaps of 0-2 ids between sends)
    gaps = rng.integers(0, 3, n)
    ours, ref = np.zeros(n, dtype=np.uint64), np.zeros(n, dtype=np.uint64)
    c_ours, c_ref = np.zeros(H, dtype=np.uint64), np.zeros(H, dtype=np.uint64)
    for i in range(n):
        s = src[i]
        c_ours[s] += gaps[i]
        c_ref[s] += gaps[i]
        ours[i] = c_ours[s]
        c_ours[s] += 1
        if kept[i]:
            ref[i] = c_ref[s]
            c_ref[s] += 1
    pa, pb = pk.copy(), pk.copy()
    pa["seq"], pb["seq"] = ours, ref
    results = []
    for p in (pa, pb):
        o = O.OracleTopology(gml)
        ips_o, _, _ = scenario.register_hosts(o, H, seed=1)
        results.append(o.round(ips_o, p, 110_000_000, 150_000_000))
    (oa, sa, ma), (ob, sb, mb) = results
    assert np.array_equal(sa, sb) and ma == mb
    assert np.array_equal(oa["pkt_index"], ob["pkt_index"])  # the same delivered order
    assert not np.array_equal(oa["seq"], ob["seq"])            # with different absolute ids
    # the ids decided real ties: some (time, dst, src) groups hold several events
    key = np.stack([oa["time"], oa["dst_host"], oa["src_host"]], 1)
    assert len(np.unique(key, axis=0)) < len(oa)
