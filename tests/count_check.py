"""Path packet counter checks (topology_incrementPathPacketCounter, worker.c:551,
counted on the device by the round kernels) shared by the GPU tests.

TEST INFRASTRUCTURE.  Two independent expectations:
  * expected_counts -- a numpy restatement over the round's own records:
    every kept packet (status delivered or end-dropped) adds 1 at its
    answering pair (owner row = the endpoint row touched first; with rows
    touched in slot order, the lower slot);
  * the oracle's own per-path counters (orc_round counts every kept packet,
    oracle.c), compared host pair by host pair.
"""
import numpy as np

KEPT = (1, 2)  # SHD_DELIVERED, SHD_DROPPED_END


def slot_map(verts):
    """host -> table slot (slots = attached vertices, ascending)."""
    sv = np.unique(verts)
    slot_of_vertex = np.full(int(sv.max()) + 1, -1, dtype=np.int64)
    slot_of_vertex[sv] = np.arange(len(sv))
    return slot_of_vertex[np.asarray(verts)]


def expected_counts(hslot, pk, status, A, touch=None):
    """Dense A x A counts of the kept packets of one round.  touch: per slot
    touch sequence (default: slot order)."""
    kept = np.isin(status, KEPT)
    s = hslot[pk["src_host"][kept]]
    d = hslot[pk["dst_host"][kept]]
    ts = s if touch is None else touch[s]
    td = d if touch is None else touch[d]
    swap = (s != d) & (td < ts)
    oi, oj = np.where(swap, d, s), np.where(swap, s, d)
    return np.bincount(oi * A + oj, minlength=A * A).reshape(A, A).astype(np.uint64)


def pair_counts(C, hslot, a, b):
    """The count of the cached path between hosts a and b read off the dense
    counters C (the pair's path is (sa, sb) or (sb, sa), never both)."""
    sa, sb = hslot[np.asarray(a)], hslot[np.asarray(b)]
    return np.where(sa == sb, C[sa, sa], C[sa, sb] + C[sb, sa])


def check_against_oracle(C, hslot, orc, ips, a, b):
    """C (summed over ranks if sharded) against the oracle's per-path counters
    for host pairs (a[k], b[k])."""
    got = pair_counts(C, hslot, a, b)
    want = np.array([orc.packet_count(int(ips[x]), int(ips[y])) for x, y in zip(a, b)], dtype=np.uint64)
    bad = np.flatnonzero(got != want)
    assert len(bad) == 0, f"{len(bad)} of {len(a)} pairs differ, first {[(int(a[i]), int(b[i])) for i in bad[:5]]}"


def expected_keys(hslot, pk, status, A, touch=None):
    """Sparse form of expected_counts: (flat pair keys, counts), keys ascending."""
    kept = np.isin(status, KEPT)
    s = hslot[pk["src_host"][kept]].astype(np.int64)
    d = hslot[pk["dst_host"][kept]].astype(np.int64)
    ts = s if touch is None else touch[s]
    td = d if touch is None else touch[d]
    swap = (s != d) & (td < ts)
    oi, oj = np.where(swap, d, s), np.where(swap, s, d)
    return np.unique(oi * A + oj, return_counts=True)


def check_rows(top, keys, counts, A, rows):
    """The product's counters of table rows `rows` (each read whole) against
    sparse expected (keys, counts): equal where expected, zero elsewhere."""
    for r in rows:
        got = top.path_packet_counts(int(r), int(r) + 1)[0]
        want = np.zeros(A, dtype=np.uint64)
        lo, hi = np.searchsorted(keys, [r * A, (r + 1) * A])
        want[keys[lo:hi] - r * A] = counts[lo:hi]
        bad = np.flatnonzero(got != want)
        assert len(bad) == 0, f"row {r}: {len(bad)} counters differ, first cols {bad[:5]}"
