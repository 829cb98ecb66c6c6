"""Host registration exactly as Shadow performs it before the first round.

Seed chain: controller Random(seed) ->
managerSeed = nextUInt (controller.c:353) -> manager Random -> schedulerSeed =
nextUInt (manager.c:199) -> per host, in registration (BTreeMap name) order,
nodeSeed = nextUInt (manager.c:344) -> host Random(nodeSeed) (host.c:164) ->
topology_attach consumes its draw (host.c:187-190, topology.c:2189).
Host ids are dense registration indices; IPs are 11.0.0.1, 11.0.0.2, ...
"""
from __future__ import annotations

import numpy as np

from .synth import host_ips


def _rand_r(state: int) -> tuple[int, int]:
    nxt = state
    nxt = (nxt * 1103515245 + 12345) & 0xFFFFFFFF
    r = (nxt >> 16) % 2048
    nxt = (nxt * 1103515245 + 12345) & 0xFFFFFFFF
    r = (r << 10) ^ ((nxt >> 16) % 1024)
    nxt = (nxt * 1103515245 + 12345) & 0xFFFFFFFF
    r = (r << 10) ^ ((nxt >> 16) % 1024)
    return r, nxt


def next_uint(state: int) -> tuple[int, int]:
    """random_nextUInt (random.c:45-51): (uint)(nextDouble * UINT_MAX)."""
    r, s = _rand_r(state)
    return int((r / 2147483647.0) * 4294967295.0), s


def host_seeds(seed: int, nhosts: int) -> np.ndarray:
    manager_seed, _ = next_uint(seed)
    ms = manager_seed
    _sched, ms = next_uint(ms)
    out = np.empty(nhosts, dtype=np.uint32)
    for h in range(nhosts):
        out[h], ms = next_uint(ms)
    return out


def register_hosts(topology, nhosts: int, seed: int = 1):
    """Attaches hosts 0..nhosts-1 (no hints) to `topology` (product Topology or
    the test oracle: anything with attach(host_id, ip, rng_state)).  Returns
    (ips, rng_states_after_attach, vertices)."""
    ips = host_ips(nhosts)
    seeds = host_seeds(seed, nhosts)
    states = np.empty(nhosts, dtype=np.uint32)
    verts = np.empty(nhosts, dtype=np.int32)
    for h in range(nhosts):
        v, st, _, _ = topology.attach(h, int(ips[h]), int(seeds[h]))
        states[h] = st
        verts[h] = v
    return ips, states, verts
