"""Test infrastructure only: a pure-Python restatement of the reference's
routing/dns.c (dns_new :294-305, _dns_isIPInRange :40-87, _dns_isRestricted
:89-106, _dns_isIPUnique :108-111, _dns_generateIP :113-123, dns_register
:125-163, dns_deregister :165-181, the resolvers :183-203, the hosts file
:231-290) and address_stringToIP (address.c:145-152), with dicts in the
role of the glib hash tables.  Only tests/ may import it.

Parity pin: the reference ships no DNS test or fixture; the known answers in
tests/test_dns_cpu.py are worked by hand from the code above."""
import ipaddress
import socket
import struct

RESERVED = ["0.0.0.0/8", "10.0.0.0/8", "100.64.0.0/10", "127.0.0.0/8", "169.254.0.0/16", "172.16.0.0/12",
            "192.0.0.0/29", "192.0.2.0/24", "192.88.99.0/24", "192.168.0.0/16", "198.18.0.0/15", "198.51.100.0/24",
            "203.0.113.0/24", "224.0.0.0/4", "240.0.0.0/4", "255.255.255.255/32"]


def string_to_ip(s):
    """inet_pton into a network-order u32 (read little-endian, as the C
    in_addr_t), INADDR_NONE when unparsable."""
    try:
        return struct.unpack("<I", socket.inet_pton(socket.AF_INET, s))[0]
    except OSError:
        return 0xFFFFFFFF


def htonl(x):
    return struct.unpack("<I", struct.pack(">I", x & 0xFFFFFFFF))[0]


def ntohl(x):
    return htonl(x)


def is_in_range(net_ip, cidr):
    mask, sub = _mask_of(cidr)
    return (net_ip & mask) == sub


def _mask_of(cidr):
    sub, bits = cidr.split("/")
    bits = int(bits)
    mask = 0
    for i in range(32):
        mask = (mask << 1) & 0xFFFFFFFF
        if bits > i:
            mask += 1
    mask = htonl(mask)
    return mask, string_to_ip(sub) & mask


_MASKS = [_mask_of(c) for c in RESERVED]  # is_in_range's (mask, subnet) per block, computed once


def is_restricted(net_ip):
    return any((net_ip & m) == s for m, s in _MASKS)


class OracleDns:
    def __init__(self):
        self.ip_counter = ntohl(string_to_ip("11.0.0.0"))
        self.mac_counter = 0
        self.by_ip = {}
        self.by_name = {}

    def _generate(self):
        self.ip_counter += 1
        ip = htonl(self.ip_counter)
        while is_restricted(ip) or ip in self.by_ip:
            self.ip_counter += 1
            ip = htonl(self.ip_counter)
        return ip

    def register(self, name, requested_ip=None):
        self.mac_counter += 1
        mac = self.mac_counter
        local = False
        if requested_ip is not None:
            ip = string_to_ip(requested_ip)
            if ip == string_to_ip("127.0.0.1"):
                local = True
            elif is_restricted(ip) or ip in self.by_ip:
                ip = self._generate()
        else:
            ip = self._generate()
        if not local:
            addr = (ip, mac, name)
            self.by_ip[ip] = addr
            self.by_name[name] = addr
        return ip, mac, local

    def deregister(self, ip, name, is_local=False):
        if not is_local:
            self.by_ip.pop(ip, None)
            self.by_name.pop(name, None)

    def resolve_ip(self, ip):
        a = self.by_ip.get(ip)
        return None if a is None else (a[2], a[1])

    def resolve_name(self, name):
        a = self.by_name.get(name)
        return None if a is None else (a[0], a[1])

    def hosts_lines(self):
        """The hosts file's lines as a set (the reference's order is glib's)."""
        out = {"127.0.0.1 localhost"}
        for name, (ip, _, _) in self.by_name.items():
            out.add(f"{ipaddress.IPv4Address(struct.pack('<I', ip))} {name}")
        return out
