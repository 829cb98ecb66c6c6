"""Python mirror of Shadow's routing API (routing/topology.h:17-28) over libshdnet.

Mirrors the reference's operator interface for this path so that tests read
like the reference's call sites: ``Topology(gml, use_shortest_path)`` is
topology_new, ``attach`` is topology_attach, ``get_latency`` /
``get_reliability`` / ``is_routable`` / ``increment_path_packet_counter`` are
the lookups with their cache side effects, and the min-jump callback replaces
worker_updateMinTimeJump.  All compute runs on the GPU (HIP, gfx950).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import MINJUMP_FN, ShdError, check, lib
from .synth import DELIV_DTYPE, PKT_DTYPE

__all__ = ["Topology", "ShdError", "DeviceTable"]


def _s(x):
    return None if x is None else x.encode()


class DeviceTable:
    """A device allocation from shd_device_alloc_table (freed on close/GC).
    ``ptr`` is the device address, ``contiguous`` whether the driver granted
    physically contiguous memory."""

    def __init__(self, device: int, nbytes: int):
        p, c = C.c_void_p(), C.c_int()
        check(lib().shd_device_alloc_table(device, nbytes, C.byref(p), C.byref(c)))
        self.device, self.nbytes, self.ptr, self.contiguous = device, nbytes, p.value, bool(c.value)

    def copy_from(self, d_src_ptr: int, nbytes: int):
        assert nbytes <= self.nbytes
        check(lib().shd_device_copy(self.device, C.c_void_p(self.ptr), C.c_void_p(d_src_ptr), nbytes))

    def close(self):
        if self.ptr:
            check(lib().shd_device_free(self.device, C.c_void_p(self.ptr)))
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Topology:
    def __init__(self, gml: str, use_shortest_path: bool = True, device: int = 0, from_file: bool = False):
        self.device = device
        h = C.c_void_p()
        fn = lib().shd_topology_new if from_file else lib().shd_topology_new_from_text
        check(fn(gml.encode(), 1 if use_shortest_path else 0, device, C.byref(h)))
        self._h = h
        self._cb = None
        self.min_jump_calls: list[float] = []

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            lib().shd_topology_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def info(self):
        v, e, d, c, a = (C.c_int() for _ in range(5))
        check(lib().shd_topology_info(self._h, C.byref(v), C.byref(e), C.byref(d), C.byref(c), C.byref(a)))
        return {"vertices": v.value, "edges": e.value, "directed": bool(d.value), "complete": bool(c.value),
                "attached_vertices": a.value}

    # -- topology_attach / detach -------------------------------------------------
    def attach(self, host_id: int, ip: int, rng_state: int, ip_hint=None, city=None, country=None):
        """Returns (vertex, new_rng_state, bw_down_KiBps, bw_up_KiBps)."""
        st = C.c_uint32(rng_state)
        dn, up = C.c_uint64(), C.c_uint64()
        check(lib().shd_topology_attach(self._h, host_id, ip, C.byref(st), _s(ip_hint), _s(city), _s(country),
                                        C.byref(dn), C.byref(up)))
        v = C.c_int()
        check(lib().shd_topology_vertex_of_host(self._h, host_id, C.byref(v)))
        return v.value, st.value, dn.value, up.value

    def detach(self, ip: int):
        check(lib().shd_topology_detach(self._h, ip))

    # -- routing table ------------------------------------------------------------
    def build_routes(self):
        check(lib().shd_topology_build_routes(self._h))

    def slot_count(self) -> int:
        a = C.c_int()
        check(lib().shd_topology_slot_count(self._h, C.byref(a)))
        return a.value

    def table(self):
        """(lat_ms[A,A], rel[A,A], slot_vertex[A]) copied from the device table."""
        A = self.slot_count()
        lat = np.empty((A, A), dtype=np.float64)
        rel = np.empty((A, A), dtype=np.float64)
        sv = np.empty(A, dtype=np.int32)
        check(lib().shd_topology_copy_table(self._h, lat.ctypes.data, rel.ctypes.data, sv.ctypes.data, A))
        return lat, rel, sv

    def alloc_table(self, nbytes: int) -> "DeviceTable":
        """Device memory for a caller-owned table, allocated as the library
        allocates its own (shd_device_alloc_table)."""
        return DeviceTable(self.device, nbytes)

    def build_rows_device(self, row_lo: int, row_hi: int, d_table_ptr: int):
        check(lib().shd_topology_build_rows_device(self._h, row_lo, row_hi, C.c_void_p(d_table_ptr)))

    def latency_table_fw(self, d_lat_ptr: int, stream: int = 0):
        """The A x A latency column by blocked min-plus Floyd-Warshall into
        device memory (A*A doubles); whole-ms graphs only.  stream 0:
        synchronous; else enqueued on that hipStream_t."""
        check(lib().shd_topology_latency_table_fw(self._h, C.c_void_p(d_lat_ptr), C.c_void_p(stream)))

    def latency_rows_frontier(self, row_lo: int, row_hi: int, d_lat_ptr: int, stream: int = 0):
        """Rows [row_lo, row_hi) of the latency column by the bucketed frontier
        SSSP into device memory ((row_hi - row_lo) * A doubles); whole-ms
        graphs only; synchronous."""
        check(lib().shd_topology_latency_rows_frontier(self._h, row_lo, row_hi, C.c_void_p(d_lat_ptr),
                                                       C.c_void_p(stream)))

    def adopt_table_device(self, d_table_ptr: int):
        check(lib().shd_topology_adopt_table_device(self._h, C.c_void_p(d_table_ptr)))

    def adopt_table_device_resident(self, d_table_ptr: int):
        """Adopt without a host mirror; rows are released lazily by the
        lookups and sends that first touch them (touch_all: steady state)."""
        check(lib().shd_topology_adopt_table_device_resident(self._h, C.c_void_p(d_table_ptr)))

    @staticmethod
    def _shard_args(devices, d_rows, row_bounds):
        n = len(devices)
        assert len(d_rows) == n and len(row_bounds) == n + 1
        return (n, (C.c_int * n)(*[int(x) for x in devices]), (C.c_void_p * n)(*[int(x) for x in d_rows]),
                (C.c_int * (n + 1))(*[int(x) for x in row_bounds]))

    def build_shards(self, devices, d_rows, row_bounds):
        """Rows [row_bounds[k], row_bounds[k+1]) into d_rows[k] on devices[k], shards concurrently."""
        check(lib().shd_topology_build_shards(self._h, *self._shard_args(devices, d_rows, row_bounds)))

    def adopt_table_shards(self, devices, d_rows, row_bounds):
        """Single-process multi-GPU table: one release state over the shards."""
        check(lib().shd_topology_adopt_table_shards(self._h, *self._shard_args(devices, d_rows, row_bounds)))

    def set_host_bounds(self, host_bounds):
        hb = (C.c_uint32 * len(host_bounds))(*[int(x) for x in host_bounds])
        check(lib().shd_topology_set_host_bounds(self._h, hb))

    def touch_all(self):
        check(lib().shd_topology_touch_all(self._h))

    # -- lookups (topology_getLatency & co, with the cache side effects) -----------
    def get_latency(self, src_ip: int, dst_ip: int) -> float:
        out = C.c_double()
        check(lib().shd_topology_get_latency(self._h, src_ip, dst_ip, C.byref(out)))
        return out.value

    def get_reliability(self, src_ip: int, dst_ip: int) -> float:
        out = C.c_double()
        check(lib().shd_topology_get_reliability(self._h, src_ip, dst_ip, C.byref(out)))
        return out.value

    def is_routable(self, src_ip: int, dst_ip: int) -> bool:
        out = C.c_int()
        check(lib().shd_topology_is_routable(self._h, src_ip, dst_ip, C.byref(out)))
        return bool(out.value)

    def lookup_batch(self, src_ips, dst_ips):
        """n getLatency lookups in order (side effects included): (lat_ms[n], rel[n])."""
        s = np.ascontiguousarray(src_ips, dtype=np.uint32)
        d = np.ascontiguousarray(dst_ips, dtype=np.uint32)
        lat = np.empty(len(s), dtype=np.float64)
        rel = np.empty(len(s), dtype=np.float64)
        check(lib().shd_topology_lookup_batch(self._h, s.ctypes.data, d.ctypes.data, len(s), lat.ctypes.data,
                                              rel.ctypes.data))
        return lat, rel

    def increment_path_packet_counter(self, src_ip: int, dst_ip: int):
        check(lib().shd_topology_increment_path_packet_counter(self._h, src_ip, dst_ip))

    def path_packet_count(self, src_ip: int, dst_ip: int) -> int:
        out = C.c_uint64()
        check(lib().shd_topology_get_path_packet_count(self._h, src_ip, dst_ip, C.byref(out)))
        return out.value

    def path_packet_counts(self, row_lo: int = 0, row_hi: int | None = None) -> np.ndarray:
        """Every path packet counter of table rows [row_lo, row_hi): a
        (rows, A) u64 array, entry (i, j) = packets counted at pair (i, j)."""
        A = self.slot_count()
        row_hi = A if row_hi is None else row_hi
        out = np.empty((row_hi - row_lo, A), dtype=np.uint64)
        check(lib().shd_topology_copy_path_packet_counts(self._h, row_lo, row_hi, out.ctypes.data))
        return out

    def path_counts_sync(self):
        """Adds the rounds' logged path packet counts into the device counters."""
        check(lib().shd_topology_path_counts_sync(self._h))

    def cached_paths_log(self) -> list[str]:
        """topology_free's teardown log (shd_topology_log_cached_paths)."""
        from ._lib import PATH_LOG_FN
        lines: list[str] = []
        fn = PATH_LOG_FN(lambda line, _u: lines.append(line.decode()))
        n = C.c_uint64(0)
        check(lib().shd_topology_log_cached_paths(self._h, fn, None, C.byref(n)))
        assert n.value == len(lines)
        return lines

    def min_path_latency(self) -> float:
        out = C.c_double()
        check(lib().shd_topology_get_min_path_latency(self._h, C.byref(out)))
        return out.value

    def next_min_jump_ns(self) -> int:
        """What controller_updateMinTimeJump (controller.c:141-153) holds after
        the recorded callback values: (u64)floor(last ms) x 1e6 ns, 0 if none."""
        return int(self.min_jump_calls[-1]) * 1000000 if self.min_jump_calls else 0

    def record_min_jump(self):
        """Records every worker_updateMinTimeJump value into self.min_jump_calls."""
        def cb(ms, _user):
            self.min_jump_calls.append(ms)
        self._cb = MINJUMP_FN(cb)
        check(lib().shd_topology_set_min_jump_callback(self._h, self._cb, None))

    def host_count(self) -> int:
        n = C.c_uint32()
        check(lib().shd_topology_host_count(self._h, C.byref(n)))
        return n.value

    # -- per-round packet hand-off -------------------------------------------------
    def round(self, pkts: np.ndarray, barrier: int, end_time: int, bootstrap_end: int = 0):
        """Host API: begin + append (lookup side effects) + collect.
        Returns (delivered events, dst_offsets, status, min_time)."""
        pkts = np.ascontiguousarray(pkts, dtype=PKT_DTYPE)
        n = len(pkts)
        check(lib().shd_round_begin(self._h, barrier, end_time, bootstrap_end))
        check(lib().shd_round_append(self._h, pkts.ctypes.data, n))
        out = np.zeros(max(n, 1), dtype=DELIV_DTYPE)
        H = self.host_count()
        offs = np.zeros(H + 1, dtype=np.uint32)
        status = np.zeros(max(n, 1), dtype=np.uint8)
        nout = C.c_size_t()
        mt = C.c_uint64()
        check(lib().shd_round_collect(self._h, out.ctypes.data, len(out), C.byref(nout), offs.ctypes.data,
                                      status.ctypes.data, C.byref(mt)))
        return out[:nout.value], offs, status[:n], mt.value

    def process_device(self, d_recs: int, n: int, barrier: int, end_time: int, bootstrap_end: int, d_out: int,
                       d_offsets: int, d_status: int, d_counters: int, stream: int = 0):
        check(lib().shd_round_process_device(self._h, C.c_void_p(d_recs), n, barrier, end_time, bootstrap_end,
                                             C.c_void_p(d_out), C.c_void_p(d_offsets), C.c_void_p(d_status),
                                             C.c_void_p(d_counters), C.c_void_p(stream)))

    # -- multi-GPU rounds (shadow_amd.transport) -----------------------------------
    def exchange(self, xport, d_events: int, d_offsets: int, host_bounds, d_recv: int, recv_cap: int, d_out: int,
                 d_out_offsets: int, stream: int = 0) -> int:
        """shd_round_exchange: destination-owner all-to-all + regroup; returns
        the number of events received (grouped in d_out by owned host)."""
        hb = (C.c_uint32 * len(host_bounds))(*[int(x) for x in host_bounds])
        n = C.c_size_t()
        rc = lib().shd_round_exchange(self._h, xport.handle, C.c_void_p(d_events), C.c_void_p(d_offsets), hb,
                                      C.c_void_p(d_recv), recv_cap, C.c_void_p(d_out), C.c_void_p(d_out_offsets),
                                      C.byref(n), C.c_void_p(stream))
        if getattr(xport, "error", None) is not None:
            raise xport.error
        check(rc)
        return n.value

    def process_exchange(self, xport, d_recs: int, n: int, barrier: int, end_time: int, bootstrap_end: int,
                         host_bounds, d_send: int, d_status: int, d_counters: int, d_recv: int, recv_cap: int,
                         d_out: int, d_out_offsets: int, stream: int = 0) -> int:
        """shd_round_process_exchange: decide this rank's records, group them
        unsorted as 24-B wire records, exchange them to the destinations'
        owners and merge there; returns the events this rank received."""
        hb = (C.c_uint32 * len(host_bounds))(*[int(x) for x in host_bounds])
        nout = C.c_size_t()
        rc = lib().shd_round_process_exchange(self._h, xport.handle, C.c_void_p(d_recs), n, barrier, end_time,
                                              bootstrap_end, hb, C.c_void_p(d_send), C.c_void_p(d_status),
                                              C.c_void_p(d_counters), C.c_void_p(d_recv), recv_cap, C.c_void_p(d_out),
                                              C.c_void_p(d_out_offsets), C.byref(nout), C.c_void_p(stream))
        if getattr(xport, "error", None) is not None:
            raise xport.error
        check(rc)
        return nout.value

    def route_records(self, xport, d_recs: int, n: int, row_bounds, d_scratch: int, d_recv: int, recv_cap: int,
                      stream: int = 0) -> int:
        """shd_round_route_records: each record to the rank holding its answering row."""
        rb = (C.c_uint32 * len(row_bounds))(*[int(x) for x in row_bounds])
        nr = C.c_size_t()
        rc = lib().shd_round_route_records(self._h, xport.handle, C.c_void_p(d_recs), n, rb, C.c_void_p(d_scratch),
                                           C.c_void_p(d_recv), recv_cap, C.byref(nr), C.c_void_p(stream))
        if getattr(xport, "error", None) is not None:
            raise xport.error
        check(rc)
        return nr.value

    def allgather_rows(self, xport, d_table: int, row_bounds, stream: int = 0):
        """shd_topology_allgather_rows: completes this rank's A x A table
        (rows [row_bounds[rank], row_bounds[rank+1]) built in place) with
        every other rank's rows over the transport's allgatherv."""
        rb = (C.c_uint32 * len(row_bounds))(*[int(x) for x in row_bounds])
        rc = lib().shd_topology_allgather_rows(self._h, xport.handle, C.c_void_p(d_table), rb, C.c_void_p(stream))
        if rc and getattr(xport, "error", None) is not None:
            raise xport.error
        check(rc)

    def shard_min_latency(self, d_rows: int, row_lo: int, row_hi: int) -> float:
        out = C.c_double()
        check(lib().shd_topology_shard_min_latency(self._h, C.c_void_p(d_rows), row_lo, row_hi, C.byref(out)))
        return out.value

    def adopt_table_shard_device_resident(self, d_rows: int, row_lo: int, row_hi: int, global_min_ms: float = -1.0):
        check(lib().shd_topology_adopt_table_shard_device_resident(self._h, C.c_void_p(d_rows), row_lo, row_hi,
                                                                   global_min_ms))

    def deliv_sort_device(self, d_in: int, n: int, host_lo: int, host_hi: int, d_out: int, d_offsets: int,
                          stream: int = 0):
        check(lib().shd_deliv_sort_device(self._h, C.c_void_p(d_in), n, host_lo, host_hi, C.c_void_p(d_out),
                                          C.c_void_p(d_offsets), C.c_void_p(stream)))
