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


# ---- network interfaces (shd_nic_*) -------------------------------------

NIC_STATE_DTYPE = np.dtype([("recv_remaining", "<u8"), ("recv_refill", "<u8"), ("recv_capacity", "<u8"),
                            ("send_remaining", "<u8"), ("send_refill", "<u8"), ("send_capacity", "<u8"),
                            ("refill_start", "<u8"), ("refill_time", "<u8"), ("refill_pending", "<u4"),
                            ("pad0", "<u4"), ("pad1", "<u8"), ("router", STATE_DTYPE)])
SEND_DTYPE = np.dtype([("ready", "<u8"), ("id", "<u4"), ("length", "<u4")])
NIC_QUEUED, NIC_RECEIVED, NIC_DROPPED = 0, 1, 2
NEVER = 0xFFFFFFFFFFFFFFFF
HEADER_UDP, HEADER_TCP = 42, 66  # CONFIG_HEADER_SIZE_UDPIPETH / _TCPIPETH (definitions.h:173-180)
assert NIC_STATE_DTYPE.itemsize == 128


class Interfaces:
    """Network interfaces of hosts [host_base, host_base + n): token buckets,
    refill grid and upstream CoDel router per host, resident on the device
    (host/network_interface.c + routing/router.c)."""

    def __init__(self, n: int, bw_down_kibps, bw_up_kibps, start_time: int, ring_cap: int, fate_cap: int,
                 host_base: int = 0, device="cuda"):
        self.n, self.base, self.cap, self.device = n, host_base, ring_cap, torch.device(device)
        self.states = torch.zeros(n * NIC_STATE_DTYPE.itemsize, dtype=torch.uint8, device=self.device)
        self.rings = torch.zeros(n * ring_cap * ENTRY_DTYPE.itemsize, dtype=torch.uint8, device=self.device)
        self.recv_time = torch.full((fate_cap,), -1, dtype=torch.int64, device=self.device)
        self.recv_status = torch.zeros(fate_cap, dtype=torch.uint8, device=self.device)
        self.fate_cap = fate_cap
        dn = torch.as_tensor(np.asarray(bw_down_kibps, dtype=np.uint64).view(np.int64), device=self.device)
        up = torch.as_tensor(np.asarray(bw_up_kibps, dtype=np.uint64).view(np.int64), device=self.device)
        check(lib().shd_nic_init(n, dn.data_ptr(), up.data_ptr(), start_time, self.states.data_ptr(), None))
        torch.cuda.synchronize(self.device)

    def run_device(self, d_events: int, d_offsets: int, d_lengths: int, window_end: int, bootstrap_end: int = 0,
                   id_base: int = 0, d_sends: int = 0, d_send_offsets: int = 0, d_send_time: int = 0, stream=0):
        """shd_nic_run on device buffers (raw pointers)."""
        check(lib().shd_nic_run(self.n, self.base, d_events or None, d_offsets, d_lengths or None, d_sends or None,
                                d_send_offsets or None, window_end, bootstrap_end, self.states.data_ptr(),
                                self.rings.data_ptr(), self.cap, id_base, self.recv_time.data_ptr(),
                                self.recv_status.data_ptr(), self.fate_cap, d_send_time or None, stream))

    def run(self, events: np.ndarray, offsets: np.ndarray, lengths: np.ndarray, window_end: int,
            bootstrap_end: int = 0, id_base: int = 0, sends: np.ndarray | None = None,
            send_offsets: np.ndarray | None = None):
        """Host arrays in, send times out (receive fates stay in
        recv_time / recv_status, indexed by packet id)."""
        d_ev = _dev(events, self.device) if len(events) else None
        d_off = _dev(np.asarray(offsets, dtype=np.uint32), self.device)
        d_len = _dev(np.asarray(lengths, dtype=np.uint32), self.device) if len(events) else None
        d_s = d_so = d_st = None
        if sends is not None:
            d_s = _dev(sends.astype(SEND_DTYPE), self.device) if len(sends) else torch.empty(16, dtype=torch.uint8,
                                                                                             device=self.device)
            d_so = _dev(np.asarray(send_offsets, dtype=np.uint32), self.device)
            d_st = torch.empty(max(len(sends), 1), dtype=torch.int64, device=self.device)
        torch.cuda.synchronize(self.device)
        self.run_device(d_ev.data_ptr() if d_ev is not None else 0, d_off.data_ptr(),
                        d_len.data_ptr() if d_len is not None else 0, window_end, bootstrap_end, id_base,
                        d_s.data_ptr() if d_s is not None else 0, d_so.data_ptr() if d_so is not None else 0,
                        d_st.data_ptr() if d_st is not None else 0)
        if d_st is None:
            return None
        return d_st.cpu().numpy().view(np.uint64)[:len(sends)].copy()

    def state(self) -> np.ndarray:
        return self.states.cpu().numpy().view(NIC_STATE_DTYPE).copy()

    def fates(self):
        return (self.recv_time.cpu().numpy().view(np.uint64).copy(), self.recv_status.cpu().numpy().copy())
