"""Synthetic, seeded workloads for the network plane.

Graphs are emitted as GML in the dialect Shadow reads (docs/network_graph_spec.md;
fixture src/test/config/convert/topology.expected.gml): ``directed``, ``node [ id
bandwidth_up bandwidth_down ]`` and ``edge [ source target latency packet_loss ]``.
All randomness comes from splitmix64 so that the same seed gives the same graph,
hosts and packets on every machine (build container and GPU box alike).
"""
from __future__ import annotations

import numpy as np

MASK64 = (1 << 64) - 1


class SplitMix64:
    """splitmix64 stream (seed 0x5EED0000 + config per SURVEY.md §8d)."""

    def __init__(self, seed: int):
        self.s = seed & MASK64

    def next(self) -> int:
        self.s = (self.s + 0x9E3779B97F4A7C15) & MASK64
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        return z ^ (z >> 31)

    def below(self, n: int) -> int:
        return self.next() % n

    def array(self, n: int) -> np.ndarray:
        """n draws as a uint64 array (vectorised splitmix64 over a counter)."""
        base = np.uint64(self.s)
        idx = np.arange(1, n + 1, dtype=np.uint64)
        with np.errstate(over="ignore"):
            z = base + idx * np.uint64(0x9E3779B97F4A7C15)
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            z = z ^ (z >> np.uint64(31))
            self.s = int((base + np.uint64(n) * np.uint64(0x9E3779B97F4A7C15)) & np.uint64(MASK64))
        return z


def _edge_block(a: int, b: int, latency: str, loss: float) -> str:
    return f"  edge [\n    source {a}\n    target {b}\n    latency \"{latency}\"\n    packet_loss {loss!r}\n  ]\n"


def _node_block(i: int, bw: str = "1 Gbit", ip: str | None = None) -> str:
    s = f"  node [\n    id {i}\n"
    if ip is not None:
        s += f"    ip_address \"{ip}\"\n"
    s += f"    bandwidth_up \"{bw}\"\n    bandwidth_down \"{bw}\"\n  ]\n"
    return s


def _latency_string(rng: SplitMix64, ns_variant: bool, lo_ms: int, hi_ms: int) -> str:
    if ns_variant:
        return f"{lo_ms * 100000 + rng.below((hi_ms - lo_ms) * 1000000)} ns"
    return f"{lo_ms + rng.below(hi_ms - lo_ms + 1)} ms"


def complete_graph_gml(V: int, seed: int, ns_variant: bool = False, directed: bool = False,
                       max_loss_permille: int = 50, max_ms: int = 300) -> str:
    """C1: complete graph with self-loops (Tor-style), latency 1..max_ms ms
    (or ns-resolution variant), loss k/1000 with k in [0, max_loss_permille]."""
    rng = SplitMix64(seed)
    out = [f"graph [\n  directed {1 if directed else 0}\n"]
    out += [_node_block(i) for i in range(V)]
    for a in range(V):
        for b in range((0 if directed else a), V):
            lat = _latency_string(rng, ns_variant, 1, max_ms)
            loss = rng.below(max_loss_permille + 1) / 1000.0
            out.append(_edge_block(a, b, lat, loss))
    out.append("]\n")
    return "".join(out)


def sparse_graph_gml(V: int, seed: int, avg_degree: float = 7.0, ns_variant: bool = False,
                     directed: bool = False, max_loss_permille: int = 20, max_ms: int = 150,
                     self_loops: bool = True) -> str:
    """C2/C4: "Internet-like" sparse graph: random spanning tree plus
    preferential-attachment extra edges; simple graph (no parallel edges);
    every vertex gets a self-loop (Shadow's access-link convention)."""
    rng = SplitMix64(seed)
    edges: set[tuple[int, int]] = set()
    deg = [0] * V
    ends: list[int] = []
    for v in range(1, V):
        u = rng.below(v) if (not ends or rng.below(2) == 0) else ends[rng.below(len(ends))]
        key = (min(u, v), max(u, v))
        edges.add(key)
        ends += [u, v]
        deg[u] += 1
        deg[v] += 1
    target_edges = int(V * avg_degree / 2)
    tries = 0
    while len(edges) < target_edges and tries < target_edges * 20:
        tries += 1
        a = ends[rng.below(len(ends))]
        b = rng.below(V)
        if a == b:
            continue
        key = (min(a, b), max(a, b))
        if key in edges:
            continue
        edges.add(key)
        ends += [a, b]
    out = [f"graph [\n  directed {1 if directed else 0}\n"]
    out += [_node_block(i) for i in range(V)]
    for (a, b) in sorted(edges):
        for (x, y) in ([(a, b), (b, a)] if directed else [(a, b)]):
            lat = _latency_string(rng, ns_variant, 1, max_ms)
            loss = rng.below(max_loss_permille + 1) / 1000.0
            out.append(_edge_block(x, y, lat, loss))
    if self_loops:
        for v in range(V):
            out.append(_edge_block(v, v, _latency_string(rng, ns_variant, 1, 5), 0.0))
    out.append("]\n")
    return "".join(out)


ONE_GBIT_SWITCH_GML = """graph [
  directed 0
  node [
    id 0
    ip_address "0.0.0.0"
    bandwidth_up "1 Gbit"
    bandwidth_down "1 Gbit"
  ]
  edge [
    source 0
    target 0
    latency "1 ms"
    packet_loss 0.0
  ]
]"""
"""The built-in ``1_gbit_switch`` graph (configuration.rs:728-742), C0."""


def host_ips(n: int) -> np.ndarray:
    """Network-order IPv4 addresses 11.0.0.1, 11.0.0.2, ... as Shadow's DNS
    hands them out (little-endian u32 view of the in_addr bytes)."""
    h = np.arange(n, dtype=np.uint64) + np.uint64((11 << 24) + 1)
    b0 = (h >> np.uint64(24)) & np.uint64(0xFF)
    b1 = (h >> np.uint64(16)) & np.uint64(0xFF)
    b2 = (h >> np.uint64(8)) & np.uint64(0xFF)
    b3 = h & np.uint64(0xFF)
    return (b0 | (b1 << np.uint64(8)) | (b2 << np.uint64(16)) | (b3 << np.uint64(24))).astype(np.uint32)


def glibc_rand_r_advance(states: np.ndarray) -> np.ndarray:
    """One glibc rand_r step on a vector of states (state update only)."""
    s = states.astype(np.uint64)
    for _ in range(3):
        s = (s * np.uint64(1103515245) + np.uint64(12345)) & np.uint64(0xFFFFFFFF)
    return s.astype(np.uint32)


PKT_DTYPE = np.dtype([("now", "<u8"), ("seq", "<u8"), ("src_host", "<u4"), ("dst_host", "<u4"),
                      ("rng_state", "<u4"), ("payload_len", "<u4")])
DELIV_DTYPE = np.dtype([("time", "<u8"), ("seq", "<u8"), ("src_host", "<u4"), ("dst_host", "<u4"),
                        ("pkt_index", "<u4"), ("pad", "<u4")])


def packet_batch(n: int, nhosts: int, seed: int, window_start: int, window_ns: int,
                 host_seeds: np.ndarray, zipf: bool = False, p_payload: float = 0.9,
                 hosts_lo: int = 0, hosts_hi: int | None = None, hosts: np.ndarray | None = None,
                 pairs: tuple[np.ndarray, np.ndarray] | None = None) -> np.ndarray:
    """C3: one round's packet records.  src uniform over [hosts_lo, hosts_hi)
    (or Zipf: zipf=True the log-uniform s=1 form, zipf=1.1 Zipf(1.1) ranks,
    host hosts_lo the most frequent), dst uniform != src over all hosts, now uniform in the
    window, payload 1448 B with prob p_payload else 0.  With `hosts` given,
    src and dst are both drawn from that host list instead (bounded samples);
    with `pairs` = (src, dst) arrays of length n they are taken as given.
    rng_state = the src host's real rand_r state advanced once per earlier
    packet of that host in this batch (the CPU reserves one draw per send);
    seq = per-src ordinal."""
    rng = SplitMix64(seed)
    r = rng.array(4 * n)
    if pairs is not None:
        src = np.asarray(pairs[0], dtype=np.uint32)
        dst = np.asarray(pairs[1], dtype=np.uint32)
        assert len(src) == len(dst) == n
    elif hosts is not None:
        hosts = np.asarray(hosts, dtype=np.uint32)
        m = len(hosts)
        si = (r[0::4] % np.uint64(m)).astype(np.int64)
        di = (r[1::4] % np.uint64(m - 1)).astype(np.int64)
        di = np.where(di >= si, di + 1, di)
        src, dst = hosts[si], hosts[di]
    else:
        hi = nhosts if hosts_hi is None else hosts_hi
        span = hi - hosts_lo
        if zipf:
            u = (r[0::4] >> np.uint64(11)).astype(np.float64) / float(1 << 53)
            if zipf is True or float(zipf) == 1.0:
                ranks = np.floor(np.power(span, u)).astype(np.int64)  # log-uniform ~ Zipf(1)
            else:  # Zipf(s): inverse CDF of the continuous density x^-s on [1, span + 1)
                e = 1.0 - float(zipf)
                ranks = np.floor(np.power(1.0 + u * (np.power(span + 1.0, e) - 1.0), 1.0 / e)).astype(np.int64)
            src = (hosts_lo + np.clip(ranks - 1, 0, span - 1)).astype(np.uint32)
        else:
            src = (hosts_lo + (r[0::4] % np.uint64(span))).astype(np.uint32)
        dst = (r[1::4] % np.uint64(nhosts - 1)).astype(np.uint32)
        dst = np.where(dst >= src, dst + 1, dst).astype(np.uint32)
    now = np.uint64(window_start) + (r[2::4] % np.uint64(window_ns))
    payload = np.where((r[3::4] % np.uint64(1000)) < np.uint64(int(p_payload * 1000)), 1448, 0).astype(np.uint32)
    # per-src ordinal (stable in batch order)
    order = np.argsort(src, kind="stable")
    ss = src[order]
    starts = np.r_[0, np.flatnonzero(np.diff(ss)) + 1]
    runlen = np.diff(np.r_[starts, len(ss)])
    ordinal_sorted = np.arange(len(ss)) - np.repeat(starts, runlen)
    ordinal = np.empty(n, dtype=np.int64)
    ordinal[order] = ordinal_sorted
    # rng pre-state: host seed advanced `ordinal` times
    # one rand_r draw = three LCG steps = an affine map s -> a*s + c (mod 2^32);
    # k draws = (A_k, C_k), so the pre-state is a single gather + FMA.
    maxo = int(ordinal.max()) if n else 0
    a1, c1 = 1, 0
    for _ in range(3):
        a1, c1 = (a1 * 1103515245) & 0xFFFFFFFF, (c1 * 1103515245 + 12345) & 0xFFFFFFFF
    A = np.empty(maxo + 1, dtype=np.uint64)
    C = np.empty(maxo + 1, dtype=np.uint64)
    ak, ck = 1, 0
    for k in range(maxo + 1):
        A[k], C[k] = ak, ck
        ak, ck = (a1 * ak) & 0xFFFFFFFF, (a1 * ck + c1) & 0xFFFFFFFF
    s0 = host_seeds[src].astype(np.uint64)
    pre = ((A[ordinal] * s0 + C[ordinal]) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    rec = np.empty(n, dtype=PKT_DTYPE)
    rec["now"] = now
    rec["seq"] = ordinal.astype(np.uint64)
    rec["src_host"] = src
    rec["dst_host"] = dst
    rec["rng_state"] = pre
    rec["payload_len"] = payload
    return rec


def redraw_destinations(rec: np.ndarray, nhosts: int, seed: int) -> np.ndarray:
    """A copy of a packet batch with new uniform destinations (!= src): the
    same senders, send times, per-src ordinals and rand_r pre-states (they
    depend on the sender alone), so a valid round whose table gathers are
    other lines than the original's -- fresh inputs for timed rounds,
    ~20x cheaper than a new packet_batch at 10M."""
    out = rec.copy()
    src = rec["src_host"]
    dst = (SplitMix64(seed).array(len(rec)) % np.uint64(nhosts - 1)).astype(np.uint32)
    out["dst_host"] = np.where(dst >= src, dst + 1, dst).astype(np.uint32)
    return out


def _mix64(z: np.ndarray) -> np.ndarray:
    """splitmix64's finaliser on a uint64 array (csrc/synth.hip mix64)."""
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def synth_sends(pool: np.ndarray, m: int, rnd: int, seed: int, t0: int, window_ns: int, states: np.ndarray,
                seqs: np.ndarray, dst_pool: np.ndarray | None = None, ndst: int | None = None):
    """numpy restatement of shd_synth_sends_device (csrc/synth.hip), the
    simulated rounds' load generator: sender k = pool[k] sends m packets;
    packet j reserves the sender's j-th rand_r draw of the round (its record
    carries the pre-state; the state m draws on is carried out), goes to a
    hashed destination (dst_pool[x % ndst], or host x % ndst; the next one if
    that is the sender itself) at a time in the j-th of m slices of [t0, t0 +
    window).  Returns (records, states after the round, seqs after)."""
    pool = np.asarray(pool, dtype=np.uint32)
    npool = len(pool)
    n = npool * m
    ndst = len(dst_pool) if dst_pool is not None else int(ndst)
    with np.errstate(over="ignore"):
        key = np.uint64(seed) * np.uint64(0xD1B54A32D192ED03) + np.uint64(rnd) * np.uint64(0x8CB92BA72F3D8DD7)
        x = _mix64(key + np.arange(n, dtype=np.uint64))
    k = np.repeat(np.arange(npool), m)
    j = np.tile(np.arange(m, dtype=np.uint64), npool)
    h = pool[k]
    s = np.asarray(states, dtype=np.uint32)[k]
    st = s.copy()
    for step in range(1, m):  # packet j's pre-state: j draws into the round
        s = glibc_rand_r_advance(s)
        st = np.where(j >= np.uint64(step), s, st)
    di = (x % np.uint64(ndst)).astype(np.int64)
    dmap = (lambda i: np.asarray(dst_pool, dtype=np.uint32)[i]) if dst_pool is not None else \
        (lambda i: i.astype(np.uint32))
    d = dmap(di)
    clash = (d == h) & (ndst > 1)
    di = np.where(clash, np.where(di + 1 == ndst, 0, di + 1), di)
    d = dmap(di)
    sl = np.uint64(window_ns // m)
    rec = np.empty(n, dtype=PKT_DTYPE)
    rec["now"] = np.uint64(t0) + j * sl + ((x >> np.uint64(32)) % sl if int(sl) else np.uint64(0))
    rec["seq"] = np.asarray(seqs, dtype=np.uint64)[k] + j
    rec["src_host"] = h
    rec["dst_host"] = d
    rec["rng_state"] = st
    rec["payload_len"] = np.where(((x >> np.uint64(16)) & np.uint64(1023)) < np.uint64(922), 1448, 0).astype(np.uint32)
    out_states = np.asarray(states, dtype=np.uint32).copy()
    for _ in range(m):
        out_states = glibc_rand_r_advance(out_states)
    return rec, out_states, np.asarray(seqs, dtype=np.uint64) + np.uint64(m)
