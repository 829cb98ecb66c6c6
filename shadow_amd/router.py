"""Destination routers with CoDel (include/shdnet.h ``shd_codel_run``).

Host mirror of routing/router.c:103-131 (router_enqueue / router_dequeue) and
routing/router_queue_codel.c:113-265 for the step that follows the packet
hand-off: every destination host's upstream router.  ``CodelRouters`` keeps
one state record and one entry ring per router resident on the device; a
batch of operations (enqueue at a packet's arrival, dequeue when the
receiving interface pulls) runs for all routers at once, and packets still
queued carry over to the next batch.
"""
from __future__ import annotations

import numpy as np
import torch

from ._lib import check, lib

STATE_DTYPE = np.dtype([("interval_expire", "<u8"), ("next_drop", "<u8"), ("total_size", "<u8"), ("mode", "<u4"),
                        ("drop_count", "<u4"), ("drop_count_last", "<u4"), ("head", "<u4"), ("len", "<u4"),
                        ("pad", "<u4")])
ENTRY_DTYPE = np.dtype([("enqueue_ts", "<u8"), ("pkt", "<u4"), ("length", "<u4")])
OP_DTYPE = np.dtype([("time", "<u8"), ("kind", "<u4"), ("pkt", "<u4"), ("length", "<u4"), ("pad", "<u4")])
ENQUEUE, DEQUEUE = 0, 1
QUEUED, DEQUEUED, DROPPED = 0, 1, 2
NO_PACKET = 0xFFFFFFFF
assert STATE_DTYPE.itemsize == 48 and ENTRY_DTYPE.itemsize == 16 and OP_DTYPE.itemsize == 24


def _dev(a: np.ndarray, device) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8)).to(device)


class CodelRouters:
    """``nrouters`` CoDel routers with rings of ``ring_cap`` entries each (the
    reference queue is unbounded; a ring that would overflow fails the batch
    with -ENOSPC instead of dropping)."""

    def __init__(self, nrouters: int, ring_cap: int, device="cuda"):
        self.n, self.cap, self.device = nrouters, ring_cap, torch.device(device)
        self.states = torch.zeros(nrouters * STATE_DTYPE.itemsize, dtype=torch.uint8, device=self.device)
        self.rings = torch.zeros(nrouters * ring_cap * ENTRY_DTYPE.itemsize, dtype=torch.uint8, device=self.device)

    def run(self, op_offsets: np.ndarray, ops: np.ndarray, npkts: int, stream=0):
        """Runs ops[op_offsets[r]:op_offsets[r+1]] on router r (times
        non-decreasing per router).  Returns (deq_out, fate): per op the
        packet enqueued / dequeued (NO_PACKET for an empty dequeue), and per
        packet id < npkts ``(op index << 2) | status`` of its last event
        (all-ones if the batch did not touch it)."""
        assert len(op_offsets) == self.n + 1 and op_offsets[-1] == len(ops)
        if len(ops):
            assert ops["pkt"][ops["kind"] == ENQUEUE].max(initial=0) < npkts
        d_off = _dev(op_offsets.astype(np.uint32), self.device)
        d_ops = _dev(ops.astype(OP_DTYPE), self.device)
        deq = torch.empty(max(len(ops), 1), dtype=torch.int32, device=self.device)
        fate = torch.full((max(npkts, 1),), -1, dtype=torch.int64, device=self.device)
        torch.cuda.synchronize(self.device)
        check(lib().shd_codel_run(self.n, d_off.data_ptr(), d_ops.data_ptr(), self.states.data_ptr(),
                                  self.rings.data_ptr(), self.cap, deq.data_ptr(), fate.data_ptr(), stream))
        return (deq.cpu().numpy().view(np.uint32)[:len(ops)].copy(),
                fate.cpu().numpy().view(np.uint64)[:npkts].copy())

    def state(self) -> np.ndarray:
        return self.states.cpu().numpy().view(STATE_DTYPE).copy()

    def queued(self, r: int) -> np.ndarray:
        """Entries still queued at router r, head first."""
        st = self.state()[r]
        ring = self.rings.view(-1)[r * self.cap * 16:(r + 1) * self.cap * 16].cpu().numpy().view(ENTRY_DTYPE)
        return ring[(int(st["head"]) + np.arange(int(st["len"]))) % self.cap].copy()


def trace_from_arrivals(router: np.ndarray, arrival: np.ndarray, length: np.ndarray, nrouters: int,
                        service_ns_per_byte: float):
    """Synthetic router operations for packets arriving at ``router[i]`` at
    ``arrival[i]`` (grouped by router, non-decreasing per router): an enqueue
    at the arrival and a dequeue when a receiver serving one packet at a time
    at ``service_ns_per_byte`` would pull the next one (d_i = max(a_i,
    d_{i-1}) + s_i).  The receiving interface itself is not modelled; this
    is a load pattern, not networkinterface.c.  Returns (op_offsets, ops)."""
    n = len(router)
    router = np.asarray(router, dtype=np.int64)
    a = np.asarray(arrival, dtype=np.int64)
    s = np.maximum(1, np.round(np.asarray(length, dtype=np.float64) * service_ns_per_byte)).astype(np.int64)
    d = np.empty(n, dtype=np.int64)
    if n:
        # d_i = S_i + max_{j<=i}(a_j - S_{j-1}) over each router's run, S = running service sum
        start = np.r_[True, router[1:] != router[:-1]]
        seg = np.cumsum(start) - 1
        S = np.cumsum(s)
        base = np.where(start, S - s, 0)
        base = np.maximum.accumulate(np.where(start, base, -1))
        S = S - base  # per-segment running sums
        v = a - (S - s)
        big = int(v.max() - v.min() + 1)
        d = S + np.maximum.accumulate(v + seg * big) - seg * big
    ops = np.zeros(2 * n, dtype=OP_DTYPE)
    ops["time"][:n], ops["kind"][:n], ops["pkt"][:n], ops["length"][:n] = a, ENQUEUE, np.arange(n), length
    ops["time"][n:], ops["kind"][n:] = d, DEQUEUE
    r2 = np.r_[router, router]
    order = np.lexsort((ops["kind"], ops["time"], r2))
    ops = ops[order]
    off = np.zeros(nrouters + 1, dtype=np.uint32)
    np.cumsum(np.bincount(r2, minlength=nrouters), out=off[1:])
    return off, ops
