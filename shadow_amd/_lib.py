"""Loader for libshdnet.so (the in-tree HIP/C build) with ctypes prototypes.

There is deliberately no fallback: if the shared library is missing or no
gfx950 device is usable, the calls raise.  Build with ``python
__graft_entry__.py`` or ``make -C shadow_amd/csrc``.
"""
from __future__ import annotations

import ctypes as C
import errno
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# SHD_LIB: another in-tree build of the same library (A/B measurements)
LIB_PATH = os.environ.get("SHD_LIB") or os.path.join(HERE, "libshdnet.so")


class ShdError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{errno.errorcode.get(-code, code)} ({code}): {msg}")
        self.code = code


_lib = None

MINJUMP_FN = C.CFUNCTYPE(None, C.c_double, C.c_void_p)

_P = C.c_void_p
_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)
_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)
PATH_LOG_FN = C.CFUNCTYPE(None, C.c_char_p, C.c_void_p)

PROTOS = {
    "shd_topology_new": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.POINTER(_P)]),
    "shd_topology_new_from_text": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.POINTER(_P)]),
    "shd_topology_free": (None, [_P]),
    "shd_topology_attach": (C.c_int, [_P, C.c_uint32, C.c_uint32, _u32p, C.c_char_p, C.c_char_p, C.c_char_p,
                                      _u64p, _u64p]),
    "shd_topology_detach": (C.c_int, [_P, C.c_uint32]),
    "shd_topology_build_routes": (C.c_int, [_P]),
    "shd_topology_get_latency": (C.c_int, [_P, C.c_uint32, C.c_uint32, _dp]),
    "shd_topology_get_reliability": (C.c_int, [_P, C.c_uint32, C.c_uint32, _dp]),
    "shd_topology_is_routable": (C.c_int, [_P, C.c_uint32, C.c_uint32, _ip]),
    "shd_topology_increment_path_packet_counter": (C.c_int, [_P, C.c_uint32, C.c_uint32]),
    "shd_topology_get_path_packet_count": (C.c_int, [_P, C.c_uint32, C.c_uint32, _u64p]),
    "shd_topology_copy_path_packet_counts": (C.c_int, [_P, C.c_int, C.c_int, _P]),
    "shd_topology_path_counts_sync": (C.c_int, [_P]),
    "shd_topology_lookup_batch": (C.c_int, [_P, _P, _P, C.c_size_t, _P, _P]),
    "shd_topology_set_min_jump_callback": (C.c_int, [_P, MINJUMP_FN, _P]),
    "shd_topology_get_min_path_latency": (C.c_int, [_P, _dp]),
    "shd_topology_release_sync": (C.c_int, [_P]),
    "shd_topology_info": (C.c_int, [_P, _ip, _ip, _ip, _ip, _ip]),
    "shd_topology_vertex_of_host": (C.c_int, [_P, C.c_uint32, _ip]),
    "shd_topology_copy_table": (C.c_int, [_P, _P, _P, _P, C.c_int]),
    "shd_topology_slot_count": (C.c_int, [_P, _ip]),
    "shd_device_alloc_table": (C.c_int, [C.c_int, C.c_size_t, C.POINTER(_P), _ip]),
    "shd_device_free": (C.c_int, [C.c_int, _P]),
    "shd_device_copy": (C.c_int, [C.c_int, _P, _P, C.c_size_t]),
    "shd_topology_build_rows_device": (C.c_int, [_P, C.c_int, C.c_int, _P]),
    "shd_topology_latency_table_fw": (C.c_int, [_P, _P, _P]),
    "shd_topology_latency_rows_frontier": (C.c_int, [_P, C.c_int, C.c_int, _P, _P]),
    "shd_topology_adopt_table_device": (C.c_int, [_P, _P]),
    "shd_topology_adopt_table_device_resident": (C.c_int, [_P, _P]),
    "shd_topology_adopt_table_shards": (C.c_int, [_P, C.c_int, _P, _P, _P]),
    "shd_topology_build_shards": (C.c_int, [_P, C.c_int, _P, _P, _P]),
    "shd_topology_set_host_bounds": (C.c_int, [_P, _u32p]),
    "shd_topology_touch_all": (C.c_int, [_P]),
    "shd_topology_touch_order": (C.c_int, [_P, _P, _P, C.c_int]),
    "shd_topology_host_count": (C.c_int, [_P, _u32p]),
    "shd_round_begin": (C.c_int, [_P, C.c_uint64, C.c_uint64, C.c_uint64]),
    "shd_round_set_workers": (C.c_int, [_P, C.c_int]),
    "shd_round_append_worker": (C.c_int, [_P, C.c_int, _P, C.c_size_t]),
    "shd_round_append": (C.c_int, [_P, _P, C.c_size_t]),
    "shd_round_staged": (C.c_int, [_P, C.POINTER(C.c_size_t)]),
    "shd_round_collect": (C.c_int, [_P, _P, C.c_size_t, C.POINTER(C.c_size_t), _P, _P, _u64p]),
    "shd_host_buffer_alloc": (C.c_int, [C.c_size_t, C.POINTER(_P)]),
    "shd_host_buffer_free": (None, [_P]),
    "shd_round_process_device": (C.c_int, [_P, _P, C.c_size_t, C.c_uint64, C.c_uint64, C.c_uint64, _P, _P, _P, _P,
                                           _P]),
    "shd_deliv_sort_device": (C.c_int, [_P, _P, C.c_size_t, C.c_uint32, C.c_uint32, _P, _P, _P]),
    "shd_round_timing_enable": (C.c_int, [C.c_int]),
    "shd_round_timing_pause": (C.c_int, [C.c_int]),
    "shd_round_timing_read": (C.c_int, [_dp, C.c_int, _ip]),
    "shd_round_exchange_phases": (C.c_int, [_dp, C.c_int, _ip]),
    "shd_round_pipeline_of": (C.c_int, [C.c_uint32, C.c_size_t, _ip]),
    "shd_round_exchange": (C.c_int, [_P, _P, _P, _P, _u32p, _P, C.c_size_t, _P, _P, C.POINTER(C.c_size_t), _P]),
    "shd_round_process_exchange": (C.c_int, [_P, _P, _P, C.c_size_t, C.c_uint64, C.c_uint64, C.c_uint64, _u32p, _P,
                                             _P, _P, _P, C.c_size_t, _P, _P, C.POINTER(C.c_size_t), _P]),
    "shd_round_route_records": (C.c_int, [_P, _P, _P, C.c_size_t, _u32p, _P, _P, C.c_size_t,
                                          C.POINTER(C.c_size_t), _P]),
    "shd_topology_allgather_rows": (C.c_int, [_P, _P, _P, _u32p, _P]),
    "shd_topology_adopt_table_shard_device_resident": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_double]),
    "shd_topology_shard_min_latency": (C.c_int, [_P, _P, C.c_int, C.c_int, _dp]),
    "shd_transport_rccl_unique_id": (C.c_int, [_P]),
    "shd_transport_rccl_new": (C.c_int, [C.c_int, C.c_int, _P, C.c_int, C.POINTER(_P)]),
    "shd_transport_rccl_free": (None, [_P]),
    "shd_transport_rccl_new_all": (C.c_int, [C.c_int, _P, _P]),
    "shd_transport_local_new": (C.c_int, [C.c_int, _P]),
    "shd_transport_local_free": (None, [_P]),
    "shd_memcpy": (C.c_int, [_P, _P, C.c_size_t]),
    "shd_synth_sends_device": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64,
                                         _P, C.c_uint32, _P, _P, _P, _P, _P, _P]),
    "shd_topology_log_cached_paths": (C.c_int, [_P, PATH_LOG_FN, _P, _u64p]),
    "shd_nic_init": (C.c_int, [C.c_uint32, _P, _P, C.c_uint64, _P, _P]),
    "shd_event_lengths": (C.c_int, [_P, C.c_size_t, _P, C.c_uint32, _P, _P]),
    "shd_nic_run": (C.c_int, [C.c_uint32, C.c_uint32, _P, _P, _P, _P, _P, C.c_uint64, C.c_uint64, _P, _P, C.c_uint32,
                              C.c_uint32, _P, _P, C.c_uint64, _P, _P]),
    "shd_dns_new": (C.c_int, [C.POINTER(_P)]),
    "shd_dns_free": (None, [_P]),
    "shd_dns_register": (C.c_int, [_P, C.c_char_p, C.c_char_p, _u32p, _u32p, _ip]),
    "shd_dns_register_batch": (C.c_int, [_P, C.c_uint32, _P, _P, _P, _P, _P]),
    "shd_dns_deregister": (C.c_int, [_P, C.c_uint32, C.c_char_p, C.c_int]),
    "shd_dns_resolve_ip": (C.c_int, [_P, C.c_uint32, C.c_char_p, C.c_size_t, _u32p]),
    "shd_dns_resolve_name": (C.c_int, [_P, C.c_char_p, _u32p, _u32p]),
    "shd_dns_hosts_file": (C.c_int, [_P, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "shd_codel_run": (C.c_int, [C.c_uint32, _P, _P, _P, _P, C.c_uint32, _P, _P, _P]),
    "shd_parse_time_ns": (C.c_int, [C.c_char_p, _u64p]),
    "shd_parse_bandwidth_bits": (C.c_int, [C.c_char_p, _u64p]),
    "shd_last_error": (C.c_char_p, []),
}


def lib():
    """The loaded library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        # PyTorch-ROCm bundles its own libamdhip64.so.7.  Two HIP runtimes in
        # one process do not coexist, so when torch is present it is loaded
        # first and libshdnet binds to the same runtime (soname match).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `python __graft_entry__.py` "
                              "(no CPU fallback exists)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in PROTOS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc: int):
    if rc != 0:
        msg = lib().shd_last_error()
        raise ShdError(rc, msg.decode() if msg else "")
    return rc
