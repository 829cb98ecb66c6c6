"""DNS address assignment (libshdnet shd_dns_*, host C) against the
restatement of routing/dns.c in oracle/dns_oracle.py.  No GPU involved."""
import ipaddress
import struct
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "oracle"))
from dns_oracle import RESERVED, OracleDns, string_to_ip  # noqa: E402

from shadow_amd.dns import Dns  # noqa: E402


def ipstr(ip):
    return str(ipaddress.IPv4Address(struct.pack("<I", ip)))


def test_known_answers():
    """Worked by hand from dns.c: the counter starts after 11.0.0.0; a free,
    unreserved hint is taken as is; a reserved or taken one is replaced by
    the next generated address; 127.0.0.1 is local (not stored) but still
    takes a MAC number."""
    d = Dns()
    assert [ipstr(d.register("a", "11.0.0.2")[0])] == ["11.0.0.2"]
    ip, mac, loc = d.register("b")
    assert (ipstr(ip), mac, loc) == ("11.0.0.1", 2, False)
    assert ipstr(d.register("c")[0]) == "11.0.0.3"  # 11.0.0.2 is taken
    assert ipstr(d.register("d", "10.1.2.3")[0]) == "11.0.0.4"  # reserved
    assert ipstr(d.register("e", "11.0.0.1")[0]) == "11.0.0.5"  # taken
    assert ipstr(d.register("f", "not-an-ip")[0]) == "11.0.0.6"  # INADDR_NONE is reserved
    ip, mac, loc = d.register("g", "127.0.0.1")
    assert loc and mac == 7 and d.resolve_name("g") is None
    assert d.register("h", "99.1.2.3")[1] == 8
    assert d.resolve_name("c") == (string_to_ip("11.0.0.3"), 3)
    assert d.resolve_ip(string_to_ip("11.0.0.2")) == ("a", 1)
    # a name registered twice maps to the newer address; the older IP still resolves
    ip2, _, _ = d.register("a")
    assert ipstr(ip2) == "11.0.0.7" and d.resolve_name("a")[0] == ip2
    assert d.resolve_ip(string_to_ip("11.0.0.2")) == ("a", 1)
    # deregistering the old address drops its IP and the name's (new) mapping
    d.deregister(string_to_ip("11.0.0.2"), "a")
    assert d.resolve_ip(string_to_ip("11.0.0.2")) is None and d.resolve_name("a") is None
    assert d.resolve_ip(ip2) == ("a", 9)
    lines = d.hosts_file().splitlines()
    assert lines[0] == "127.0.0.1 localhost"
    assert set(lines[1:]) == {"11.0.0.1 b", "11.0.0.3 c", "11.0.0.4 d", "11.0.0.5 e", "11.0.0.6 f", "99.1.2.3 h"}


def test_reserved_block_edges():
    """First/last address of every reserved block and its neighbours, as
    hints: kept or replaced exactly as the oracle's CIDR arithmetic says."""
    hints = []
    for c in RESERVED:
        n = ipaddress.IPv4Network(c)
        lo, hi = int(n.network_address), int(n.broadcast_address)
        for x in (lo - 1, lo, hi, hi + 1):
            if 0 <= x < 2**32:
                hints.append(str(ipaddress.IPv4Address(x)))
    d, o = Dns(), OracleDns()
    for i, h in enumerate(hints):
        assert d.register(f"h{i}", h) == o.register(f"h{i}", h), h


def test_random_sequences_match_oracle():
    rng = np.random.default_rng(5)
    d, o = Dns(), OracleDns()
    live = []
    for i in range(6000):
        r = rng.random()
        name = f"host{int(rng.integers(0, 3000))}"
        if r < 0.08 and live:
            ip, nm, loc = live.pop(int(rng.integers(0, len(live))))
            d.deregister(ip, nm, loc)
            o.deregister(ip, nm, loc)
            continue
        if r < 0.4:
            hint = None
        elif r < 0.6:
            hint = f"11.0.{int(rng.integers(0, 40))}.{int(rng.integers(0, 256))}"  # collides with the generator
        elif r < 0.7:
            hint = str(ipaddress.IPv4Address(int(rng.integers(0, 2**32))))
        elif r < 0.75:
            hint = "127.0.0.1"
        elif r < 0.8:
            hint = "bogus"
        else:
            hint = f"{int(rng.integers(1, 255))}.{int(rng.integers(0, 256))}.0.1"
        got, want = d.register(name, hint), o.register(name, hint)
        assert got == want, (i, name, hint)
        live.append((got[0], name, got[2]))
        if i % 97 == 0:
            q = live[int(rng.integers(0, len(live)))]
            assert d.resolve_ip(q[0]) == o.resolve_ip(q[0])
            assert d.resolve_name(q[1]) == o.resolve_name(q[1])
    assert set(d.hosts_file().splitlines()) == o.hosts_lines()
    assert len(d.hosts_file().splitlines()) == len(o.hosts_lines())


def test_batch_200k_hosts_matches_oracle():
    """C4's startup: 200k hosts without hints, one batch call."""
    n = 200_000
    names = [f"h{i}" for i in range(n)]
    d = Dns()
    t0 = time.perf_counter()
    ip, mac, loc = d.register_batch(names)
    dt = time.perf_counter() - t0
    o = OracleDns()
    want = [o.register(nm) for nm in names]
    assert np.array_equal(ip, np.array([w[0] for w in want], np.uint32))
    assert np.array_equal(mac, np.arange(1, n + 1, dtype=np.uint32))
    assert not loc.any()
    assert dt < 5.0
    from shadow_amd import synth
    assert np.array_equal(ip, synth.host_ips(n))  # the workloads' addresses are DNS's
