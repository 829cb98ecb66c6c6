"""Host mirror of libshdnet's DNS (include/shdnet.h ``shd_dns_*``;
reference routing/dns.c): address assignment and name/IP resolution for the
simulated hosts."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, lib


def _b(s):
    return None if s is None else s.encode()


class Dns:
    def __init__(self):
        self._h = C.c_void_p()
        check(lib().shd_dns_new(C.byref(self._h)))

    def close(self):
        if self._h:
            lib().shd_dns_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def register(self, name: str, requested_ip: str | None = None):
        """dns_register: (ip_net, mac, is_local)."""
        ip, mac, loc = C.c_uint32(), C.c_uint32(), C.c_int()
        check(lib().shd_dns_register(self._h, name.encode(), _b(requested_ip), C.byref(ip), C.byref(mac),
                                     C.byref(loc)))
        return ip.value, mac.value, bool(loc.value)

    def register_batch(self, names, requested=None):
        n = len(names)
        nm = (C.c_char_p * n)(*[s.encode() for s in names])
        rq = None if requested is None else (C.c_char_p * n)(*[_b(s) for s in requested])
        ip = np.zeros(n, np.uint32)
        mac = np.zeros(n, np.uint32)
        loc = np.zeros(n, np.uint8)
        check(lib().shd_dns_register_batch(self._h, n, nm, rq, ip.ctypes.data, mac.ctypes.data, loc.ctypes.data))
        return ip, mac, loc.astype(bool)

    def deregister(self, ip_net: int, name: str, is_local: bool = False):
        check(lib().shd_dns_deregister(self._h, ip_net, name.encode(), int(is_local)))

    def resolve_ip(self, ip_net: int):
        """(name, mac) or None."""
        buf = C.create_string_buffer(1024)
        mac = C.c_uint32()
        rc = lib().shd_dns_resolve_ip(self._h, ip_net, buf, 1024, C.byref(mac))
        if rc == -2:
            return None
        check(rc)
        return buf.value.decode(), mac.value

    def resolve_name(self, name: str):
        """(ip_net, mac) or None."""
        ip, mac = C.c_uint32(), C.c_uint32()
        rc = lib().shd_dns_resolve_name(self._h, name.encode(), C.byref(ip), C.byref(mac))
        if rc == -2:
            return None
        check(rc)
        return ip.value, mac.value

    def hosts_file(self) -> str:
        n = C.c_size_t()
        check(lib().shd_dns_hosts_file(self._h, None, 0, C.byref(n)))
        buf = C.create_string_buffer(n.value + 1)
        check(lib().shd_dns_hosts_file(self._h, buf, n.value + 1, C.byref(n)))
        return buf.value.decode()
