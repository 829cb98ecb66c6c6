"""CoDel routers (routing/router_queue_codel.c:113-265) on the CPU oracle:
a hand-derived known answer, batch splitting, and the synthetic trace
generator.  The reference ships no CoDel test or fixture, so this row's
parity is pinned by the hand-derived trace below (worked through the
reference's code by hand, including its control law) -- otherwise
"parity unpinned"."""
import math

import numpy as np

import oracle_ctypes as O
from shadow_amd.router import DEQUEUE, DROPPED, DEQUEUED, ENQUEUE, NO_PACKET, OP_DTYPE, trace_from_arrivals

MS = 1_000_000


def _ops(rows):
    ops = np.zeros(len(rows), dtype=OP_DTYPE)
    for i, (t, kind, pkt) in enumerate(rows):
        ops[i] = (t, kind, pkt, 1500, 0)
    return ops


def _law(count, ts):  # _routerqueuecodel_controlLaw (:198-205): C round(), half away from zero
    return int(math.floor((ts + 100 * MS) / math.sqrt(count) + 0.5))


def test_codel_known_answer_drop_mode_and_control_law():
    """Ten 1500-byte packets queued at t=0, pulled at 20, 130 and 240 ms.
    20 ms: sojourn above target with 13500 B left -> interval starts (expires 120 ms).
    130 ms: interval expired -> store-mode drop of packet 1, packet 2 returned,
            drop mode with count 1, next drop at law(1, 130 ms) = 230 ms.
    240 ms: drop loop: packets 3..8 dropped as the reference's control law
            (ts + interval) / sqrt(count) moves the next drop backwards; packet
            9 leaves 0 B < MTU, so the queue is good again and 9 is returned."""
    rows = [(0, ENQUEUE, k) for k in range(10)] + [(20 * MS, DEQUEUE, 0), (130 * MS, DEQUEUE, 0),
                                                  (240 * MS, DEQUEUE, 0)]
    R = O.OracleRouters(1, 16)
    rc, deq, fate = R.run(np.array([0, 13], np.uint32), _ops(rows), 10)
    assert rc == 0
    assert list(deq[:10]) == list(range(10)) and list(deq[10:]) == [0, 2, 9]
    dropped = sorted(int(p) for p in range(10) if fate[p] & 3 == DROPPED)
    assert dropped == [1, 3, 4, 5, 6, 7, 8]
    assert fate[1] >> 2 == 11 and all(fate[p] >> 2 == 12 for p in (3, 4, 5, 6, 7, 8, 9))
    assert fate[0] == (10 << 2) | DEQUEUED and fate[2] == (11 << 2) | DEQUEUED
    st = R.states[0]
    nd = _law(1, 130 * MS)
    assert nd == 230 * MS
    for c in range(2, 8):  # drops 3..8 each reschedule while the queue stays bad (pkt 9 pop is good)
        if c <= 6:
            nd = _law(c, nd)
    assert int(st["next_drop"]) == nd
    assert (int(st["mode"]), int(st["drop_count"]), int(st["drop_count_last"])) == (0, 7, 1)
    assert int(st["total_size"]) == 0 and int(st["len"]) == 0 and int(st["interval_expire"]) == 0


def test_codel_empty_dequeue_and_errors():
    R = O.OracleRouters(2, 2)
    ops = _ops([(5, DEQUEUE, 0), (0, ENQUEUE, 0), (1, ENQUEUE, 1), (2, ENQUEUE, 2)])
    rc, deq, fate = R.run(np.array([0, 1, 4], np.uint32), ops, 3)
    assert rc == -2  # router 1 outgrows its 2-entry ring
    assert deq[0] == NO_PACKET and int(R.states[1]["len"]) == 2
    R2 = O.OracleRouters(1, 4)
    rc, *_ = R2.run(np.array([0, 2], np.uint32), _ops([(10, ENQUEUE, 0), (5, DEQUEUE, 0)]), 1)
    assert rc == -1  # dequeued before its enqueue time


def _random_trace(nr, seed, npr=40):
    rng = np.random.default_rng(seed)
    router = np.sort(rng.integers(0, nr, nr * npr))
    arr = np.zeros(len(router), np.int64)
    for r in range(nr):
        m = router == r
        arr[m] = np.sort(rng.integers(0, 400 * MS, m.sum()))
    length = rng.integers(60, 1500, len(router))
    return router, arr, length


def test_codel_batches_carry_state():
    """Running a trace in two batches (state and queued entries carried in the
    records) equals running it in one."""
    nr = 50
    router, arr, length = _random_trace(nr, 7)
    off, ops = trace_from_arrivals(router, arr, length, nr, 20_000.0)
    A = O.OracleRouters(nr, 4096)
    rc, deq_a, fate_a = A.run(off, ops, len(router))
    assert rc == 0
    assert (fate_a & 3 == DROPPED).sum() > 0, "the trace should push some routers into drop mode"
    B = O.OracleRouters(nr, 4096)
    cut = np.array([off[r] + (off[r + 1] - off[r]) // 2 for r in range(nr)], np.int64)
    first = np.concatenate([np.arange(off[r], cut[r]) for r in range(nr)])
    second = np.concatenate([np.arange(cut[r], off[r + 1]) for r in range(nr)])
    o1 = np.r_[0, np.cumsum(cut - off[:-1])].astype(np.uint32)
    o2 = np.r_[0, np.cumsum(off[1:] - cut)].astype(np.uint32)
    rc1, d1, f1 = B.run(o1, ops[first], len(router))
    rc2, d2, f2 = B.run(o2, ops[second], len(router))
    assert rc1 == rc2 == 0
    deq_b = np.empty_like(deq_a)
    deq_b[first], deq_b[second] = d1, d2
    assert np.array_equal(deq_a, deq_b)
    # fates name op indices of their own batch: map both back to the whole trace
    none = np.uint64(0xFFFFFFFFFFFFFFFF)
    fb = np.full_like(fate_a, none)
    for f, idx in ((f1, first), (f2, second)):
        m = f != none
        fb[m] = (idx[(f[m] >> np.uint64(2)).astype(np.int64)].astype(np.uint64) << np.uint64(2)) | (f[m] & np.uint64(3))
    assert np.array_equal(fate_a, fb)
    for k in STATE_KEYS:
        assert np.array_equal(A.states[k], B.states[k]), k


STATE_KEYS = ("interval_expire", "next_drop", "total_size", "mode", "drop_count", "drop_count_last", "len")


def test_trace_generator_departures():
    router, arr, length = _random_trace(8, 3, 30)
    off, ops = trace_from_arrivals(router, arr, length, 8, 25.0)
    for r in range(8):
        seg = ops[off[r]:off[r + 1]]
        assert (np.diff(seg["time"].astype(np.int64)) >= 0).all()
        m = np.where(router == r)[0]
        prev, want = -10**18, []
        for i in m:
            prev = max(int(arr[i]), prev) + max(1, round(int(length[i]) * 25.0))
            want.append(prev)
        assert sorted(seg["time"][seg["kind"] == DEQUEUE].tolist()) == want
