"""ctypes binding of oracle/liboracle.so (the CPU restatement).

TEST INFRASTRUCTURE: imported only by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg.  The product (shadow_amd/) never imports it.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "liboracle.so")


def _build():
    if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(
            os.path.join(ROOT, "oracle", "oracle.c")):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "liboracle.so"])


_build()
lib = C.CDLL(LIB_PATH)

u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)

lib.orc_nic_tie_count.restype = C.c_uint64
lib.orc_nic_tie_count.argtypes = []
lib.orc_parse_time_ns.restype = C.c_int64
lib.orc_parse_time_ns.argtypes = [C.c_char_p]
lib.orc_parse_bandwidth_bits.restype = C.c_int64
lib.orc_parse_bandwidth_bits.argtypes = [C.c_char_p]
lib.orc_rand_r.restype = C.c_int
lib.orc_rand_r.argtypes = [u32p]
lib.orc_next_double.restype = C.c_double
lib.orc_next_double.argtypes = [u32p]
lib.orc_next_uint.restype = C.c_uint32
lib.orc_next_uint.argtypes = [u32p]
lib.orc_topology_new.restype = C.c_void_p
lib.orc_topology_new.argtypes = [C.c_char_p, C.c_int]
lib.orc_topology_free.argtypes = [C.c_void_p]
for fn in ("orc_topology_vertex_count", "orc_topology_edge_count", "orc_topology_is_directed",
           "orc_topology_is_complete", "orc_topology_min_jump_updates"):
    getattr(lib, fn).restype = C.c_int
    getattr(lib, fn).argtypes = [C.c_void_p]
lib.orc_topology_attach.restype = C.c_int
lib.orc_topology_attach.argtypes = [C.c_void_p, C.c_uint32, u32p, C.c_char_p, C.c_char_p, C.c_char_p, u64p, u64p]
lib.orc_topology_detach.argtypes = [C.c_void_p, C.c_uint32]
for fn in ("orc_topology_get_latency", "orc_topology_get_reliability"):
    getattr(lib, fn).restype = C.c_double
    getattr(lib, fn).argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
lib.orc_topology_is_routable.restype = C.c_int
lib.orc_topology_is_routable.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
lib.orc_topology_increment_path_packet_counter.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
lib.orc_topology_path_packet_count.restype = C.c_uint64
lib.orc_topology_path_packet_count.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
lib.orc_topology_min_path_latency.restype = C.c_double
lib.orc_topology_min_path_latency.argtypes = [C.c_void_p]
lib.orc_controller_next_min_jump_ns.restype = C.c_uint64
lib.orc_controller_next_min_jump_ns.argtypes = [C.c_void_p]
lib.orc_compute_row.restype = C.c_int
lib.orc_compute_row.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
lib.orc_direct_path.restype = C.c_int
lib.orc_direct_row.restype = None
lib.orc_direct_row.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
lib.orc_direct_path.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]
lib.orc_vertex_of_ip.restype = C.c_int
lib.orc_vertex_of_ip.argtypes = [C.c_void_p, C.c_uint32]
lib.orc_topology_preload_table.restype = C.c_int
lib.orc_topology_preload_table.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
lib.orc_topology_preload_rows.restype = C.c_int
lib.orc_topology_preload_rows.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p,
                                          C.c_void_p]
lib.orc_round.restype = C.c_size_t
lib.orc_round.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64,
                          C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, u64p]
lib.orc_round_mt.restype = C.c_size_t
lib.orc_round_mt.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64,
                             C.c_void_p, C.c_size_t, C.c_int, C.c_void_p, C.c_void_p, u64p]
lib.orc_pq_order.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p]
lib.orc_topology_log_cached_paths.restype = C.c_size_t
lib.orc_topology_log_cached_paths.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
lib.orc_nic_init.argtypes = [C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]
lib.orc_nic_run.argtypes = [C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                            C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p,
                            C.c_void_p, C.c_uint64, C.c_void_p]
lib.orc_codel_run.argtypes = [C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                              C.c_void_p]


def _s(x):
    return None if x is None else x.encode()


class OracleTopology:
    """Mirror of topology.h's API over the oracle (addresses are network-order IPs)."""

    def __init__(self, gml: str, use_shortest_path: bool = True):
        self.h = lib.orc_topology_new(gml.encode(), 1 if use_shortest_path else 0)
        if not self.h:
            raise ValueError("invalid topology")

    def close(self):
        if self.h:
            lib.orc_topology_free(self.h)
            self.h = None

    __del__ = close

    @property
    def V(self):
        return lib.orc_topology_vertex_count(self.h)

    @property
    def directed(self):
        return bool(lib.orc_topology_is_directed(self.h))

    @property
    def complete(self):
        return bool(lib.orc_topology_is_complete(self.h))

    def attach(self, host_id, ip, rng_state, ip_hint=None, city=None, country=None):
        """Same signature as shadow_amd.Topology.attach (host_id is unused:
        the reference keys hosts by IP)."""
        st = C.c_uint32(rng_state)
        dn, up = C.c_uint64(0), C.c_uint64(0)
        v = lib.orc_topology_attach(self.h, ip, C.byref(st), _s(ip_hint), _s(city), _s(country), C.byref(dn),
                                    C.byref(up))
        return v, st.value, dn.value, up.value

    def detach(self, ip):
        lib.orc_topology_detach(self.h, ip)

    def latency(self, s, d):
        return lib.orc_topology_get_latency(self.h, s, d)

    def reliability(self, s, d):
        return lib.orc_topology_get_reliability(self.h, s, d)

    def routable(self, s, d):
        return bool(lib.orc_topology_is_routable(self.h, s, d))

    def increment(self, s, d):
        lib.orc_topology_increment_path_packet_counter(self.h, s, d)

    def packet_count(self, s, d):
        return lib.orc_topology_path_packet_count(self.h, s, d)

    def cached_paths_log(self):
        n = lib.orc_topology_log_cached_paths(self.h, None, 0)
        buf = C.create_string_buffer(n + 1)
        lib.orc_topology_log_cached_paths(self.h, buf, n + 1)
        return buf.value.decode().splitlines()

    def min_path_latency(self):
        return lib.orc_topology_min_path_latency(self.h)

    def min_jump_updates(self):
        return lib.orc_topology_min_jump_updates(self.h)

    def next_min_jump_ns(self):
        return lib.orc_controller_next_min_jump_ns(self.h)

    def vertex_of_ip(self, ip):
        return lib.orc_vertex_of_ip(self.h, ip)

    def row(self, src, targets):
        targets = np.ascontiguousarray(targets, dtype=np.int32)
        lat = np.empty(len(targets), dtype=np.float64)
        rel = np.empty(len(targets), dtype=np.float64)
        lib.orc_compute_row(self.h, int(src), targets.ctypes.data, len(targets), lat.ctypes.data, rel.ctypes.data)
        return lat, rel

    def direct_row(self, src, targets):
        """orc_direct_row: the direct paths from src to every target (-1: no edge)."""
        targets = np.ascontiguousarray(targets, dtype=np.int32)
        lat = np.empty(len(targets), dtype=np.float64)
        rel = np.empty(len(targets), dtype=np.float64)
        lib.orc_direct_row(self.h, int(src), targets.ctypes.data, len(targets), lat.ctypes.data, rel.ctypes.data)
        return lat, rel

    def direct(self, s, d):
        lat, rel = C.c_double(), C.c_double()
        rc = lib.orc_direct_path(self.h, s, d, C.byref(lat), C.byref(rel))
        return (lat.value, rel.value) if rc == 0 else (None, None)

    def preload(self, slots, lat, rel):
        slots = np.ascontiguousarray(slots, dtype=np.int32)
        lat = np.ascontiguousarray(lat, dtype=np.float64)
        rel = np.ascontiguousarray(rel, dtype=np.float64)
        lib.orc_topology_preload_table(self.h, slots.ctypes.data, len(slots), lat.ctypes.data, rel.ctypes.data)

    def preload_rows(self, rows, cols, lat, rel):
        """Full rows over the column vertices, stored as if `rows` were touched first, in order."""
        rows = np.ascontiguousarray(rows, dtype=np.int32)
        cols = np.ascontiguousarray(cols, dtype=np.int32)
        lat = np.ascontiguousarray(lat, dtype=np.float64)
        rel = np.ascontiguousarray(rel, dtype=np.float64)
        assert lat.shape == rel.shape == (len(rows), len(cols))
        lib.orc_topology_preload_rows(self.h, rows.ctypes.data, len(rows), cols.ctypes.data, len(cols),
                                      lat.ctypes.data, rel.ctypes.data)

    def rows_parallel(self, sources, targets, threads=16):
        """orc.row for many sources on a thread pool (ctypes releases the GIL;
        rows are independent).  Returns (lat[len(sources), len(targets)], rel)."""
        from concurrent.futures import ThreadPoolExecutor
        sources = [int(s) for s in sources]
        with ThreadPoolExecutor(threads) as ex:
            res = list(ex.map(lambda s: self.row(s, targets), sources))
        return np.stack([r[0] for r in res]), np.stack([r[1] for r in res])

    def round(self, host_ips, pkts, barrier, end_time, bootstrap_end=0):
        from shadow_amd.synth import DELIV_DTYPE
        host_ips = np.ascontiguousarray(host_ips, dtype=np.uint32)
        pkts = np.ascontiguousarray(pkts)
        n = len(pkts)
        out = np.zeros(n, dtype=DELIV_DTYPE)
        status = np.zeros(n, dtype=np.uint8)
        mt = C.c_uint64(0)
        k = lib.orc_round(self.h, host_ips.ctypes.data, len(host_ips), barrier, end_time, bootstrap_end,
                          pkts.ctypes.data, n, out.ctypes.data, status.ctypes.data, C.byref(mt))
        return out[:k], status, mt.value


def round_mt(orc, host_ips, pkts, barrier, end_time, threads, bootstrap_end=0):
    """orc_round_mt: the hand-off on `threads` worker threads (rows must be preloaded)."""
    from shadow_amd.synth import DELIV_DTYPE
    host_ips = np.ascontiguousarray(host_ips, dtype=np.uint32)
    pkts = np.ascontiguousarray(pkts)
    n = len(pkts)
    out = np.zeros(n, dtype=DELIV_DTYPE)
    status = np.zeros(n, dtype=np.uint8)
    mt = C.c_uint64(0)
    k = lib.orc_round_mt(orc.h, host_ips.ctypes.data, len(host_ips), barrier, end_time, bootstrap_end,
                         pkts.ctypes.data, n, threads, out.ctypes.data, status.ctypes.data, C.byref(mt))
    if k == C.c_size_t(-1).value:
        raise ValueError("a packet's path is not cached: preload the rows first")
    return out[:k], status, mt.value


class OracleRouters:
    """orc_codel_run with the same state/ring records as shadow_amd.router."""

    def __init__(self, nrouters, ring_cap):
        from shadow_amd.router import ENTRY_DTYPE, STATE_DTYPE
        self.n, self.cap = nrouters, ring_cap
        self.states = np.zeros(nrouters, dtype=STATE_DTYPE)
        self.rings = np.zeros(nrouters * ring_cap, dtype=ENTRY_DTYPE)

    def run(self, op_offsets, ops, npkts):
        op_offsets = np.ascontiguousarray(op_offsets, dtype=np.uint32)
        ops = np.ascontiguousarray(ops)
        deq = np.zeros(max(len(ops), 1), dtype=np.uint32)
        fate = np.full(max(npkts, 1), np.uint64(0xFFFFFFFFFFFFFFFF), dtype=np.uint64)
        rc = lib.orc_codel_run(self.n, op_offsets.ctypes.data, ops.ctypes.data, self.states.ctypes.data,
                               self.rings.ctypes.data, self.cap, deq.ctypes.data, fate.ctypes.data)
        return rc, deq[:len(ops)], fate[:npkts]

    def queued(self, r):
        st = self.states[r]
        ring = self.rings[r * self.cap:(r + 1) * self.cap]
        return ring[(int(st["head"]) + np.arange(int(st["len"]))) % self.cap].copy()


class OracleInterfaces:
    """orc_nic_*: the same records as shadow_amd.router.Interfaces, on the host."""

    def __init__(self, n, bw_down_kibps, bw_up_kibps, start_time, ring_cap, fate_cap, host_base=0):
        from shadow_amd.router import ENTRY_DTYPE, NIC_STATE_DTYPE
        self.n, self.base, self.cap, self.fate_cap = n, host_base, ring_cap, fate_cap
        self.states = np.zeros(n, dtype=NIC_STATE_DTYPE)
        self.rings = np.zeros(n * ring_cap, dtype=ENTRY_DTYPE)
        self.recv_time = np.full(fate_cap, np.uint64(0xFFFFFFFFFFFFFFFF), dtype=np.uint64)
        self.recv_status = np.zeros(fate_cap, dtype=np.uint8)
        dn = np.ascontiguousarray(bw_down_kibps, dtype=np.uint64)
        up = np.ascontiguousarray(bw_up_kibps, dtype=np.uint64)
        lib.orc_nic_init(n, dn.ctypes.data, up.ctypes.data, start_time, self.states.ctypes.data)

    def run(self, events, offsets, lengths, window_end, bootstrap_end=0, id_base=0, sends=None, send_offsets=None):
        from shadow_amd.router import SEND_DTYPE
        events = np.ascontiguousarray(events)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
        st = None
        sp = sop = stp = None
        if sends is not None:
            sends = np.ascontiguousarray(sends.astype(SEND_DTYPE))
            send_offsets = np.ascontiguousarray(send_offsets, dtype=np.uint32)
            st = np.zeros(max(len(sends), 1), dtype=np.uint64)
            sp, sop, stp = sends.ctypes.data, send_offsets.ctypes.data, st.ctypes.data
        rc = lib.orc_nic_run(self.n, self.base, events.ctypes.data, offsets.ctypes.data, lengths.ctypes.data, sp, sop,
                             window_end, bootstrap_end, self.states.ctypes.data, self.rings.ctypes.data, self.cap,
                             id_base, self.recv_time.ctypes.data, self.recv_status.ctypes.data, self.fate_cap, stp)
        if rc:
            raise ValueError(f"orc_nic_run: {rc}")
        return None if st is None else st[:len(sends)]


def parse_time_ns(s):
    return lib.orc_parse_time_ns(s.encode())


def parse_bandwidth_bits(s):
    return lib.orc_parse_bandwidth_bits(s.encode())


def rand_stream(seed, n, kind="double"):
    st = C.c_uint32(seed)
    f = {"double": lib.orc_next_double, "uint": lib.orc_next_uint, "rand": lib.orc_rand_r}[kind]
    return [f(C.byref(st)) for _ in range(n)]


def seed_chain(seed, nhosts):
    st = C.c_uint32(seed)
    m = lib.orc_next_uint(C.byref(st))
    ms = C.c_uint32(m)
    sched = lib.orc_next_uint(C.byref(ms))
    hosts = [lib.orc_next_uint(C.byref(ms)) for _ in range(nhosts)]
    return m, sched, hosts


def pq_order(keys):
    arr = np.zeros(len(keys), dtype=np.dtype([("time", "<u8"), ("dst", "<u4"), ("src", "<u4"), ("seq", "<u8")]))
    for i, (t, d, s, q) in enumerate(keys):
        arr[i] = (t, d, s, q)
    order = np.zeros(len(keys), dtype=np.uint32)
    lib.orc_pq_order(arr.ctypes.data, len(keys), order.ctypes.data)
    return order.tolist()
