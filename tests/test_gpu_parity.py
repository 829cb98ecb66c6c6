"""GPU parity: libshdnet (HIP, gfx950) against the CPU oracle, through the C ABI.

Bar: bit-exact for latencies, reliabilities (the oracle reproduces igraph's
tie-breaking, so products along the same path are bitwise equal; north_star's
1e-12 relative tolerance is therefore met with margin 0), delivery status,
delivery times, per-destination order and the min delivered time.
"""
import ctypes as C

import numpy as np
import pytest

import count_check
import oracle_ctypes as O
from shadow_amd import Topology, scenario, synth

pytestmark = pytest.mark.gpu

REL_TOL = 1e-12  # north_star tolerance for reliability products (we assert bitwise)


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


def make_pair(gml, H, use_sp=True, seed=1):
    top = Topology(gml, use_shortest_path=use_sp)
    ips, st, verts = scenario.register_hosts(top, H, seed)
    orc = O.OracleTopology(gml, use_sp)
    ips2, st2, verts2 = scenario.register_hosts(orc, H, seed)
    assert (verts == verts2).all() and (st == st2).all()
    top.verts = verts
    return top, orc, ips, st


GRAPHS = {
    "1_gbit_switch": (synth.ONE_GBIT_SWITCH_GML, 4),
    "complete30_ms": (synth.complete_graph_gml(30, 0x5EED0001), 90),
    "complete40_ns": (synth.complete_graph_gml(40, 0x5EED0011, ns_variant=True), 120),
    "complete25_dir": (synth.complete_graph_gml(25, 0x5EED0031, directed=True), 80),
    "sparse300_ms": (synth.sparse_graph_gml(300, 0x5EED0002), 400),
    "sparse300_ns": (synth.sparse_graph_gml(300, 0x5EED0012, ns_variant=True), 400),
    "sparse200_dir_ns": (synth.sparse_graph_gml(200, 0x5EED0022, ns_variant=True, directed=True), 300),
    "sparse5000_hbm": (synth.sparse_graph_gml(5000, 0x5EED0042), 200),  # V > 4096: HBM-slab kernel
    "sparse4500_dir_ns_hbm": (synth.sparse_graph_gml(4500, 0x5EED0052, ns_variant=True, directed=True), 150),
    # dense enough that Dijkstra's heap holds thousands of vertices: the
    # block-loaded sink and parallel shift-up cross from LDS into the slab
    "dense4400_hbm": (synth.sparse_graph_gml(4400, 0x5EED0062, avg_degree=60.0), 120),
}


@pytest.mark.parametrize("name", list(GRAPHS))
def test_routing_table_bit_exact(name):
    gml, H = GRAPHS[name]
    top, orc, _, _ = make_pair(gml, H)
    lat, rel, sv = top.table()
    for i, s in enumerate(sv):
        ol, orl = orc.row(int(s), sv)
        assert np.array_equal(bits(lat[i]), bits(ol)), (name, i)
        assert np.array_equal(bits(rel[i]), bits(orl)), (name, i)
        nz = orl != 0
        assert np.all(np.abs(rel[i][nz] - orl[nz]) <= REL_TOL * np.abs(orl[nz]))


@pytest.mark.parametrize("name", ["sparse5000_hbm", "sparse4500_dir_ns_hbm", "dense4400_hbm"])
def test_flat_slab_kernel_bit_exact(name, monkeypatch):
    """The f64 flat-slab heap (SHD_SSSP_KERNEL=slab, heap position p at
    rest[p + 1]; the default for graphs with fractional-ms latencies) forced on
    whole-ms graphs too, where the integer-key blocked heap is the default:
    same rows, bit for bit."""
    monkeypatch.setenv("SHD_SSSP_KERNEL", "slab")
    gml, H = GRAPHS[name]
    top, orc, _, _ = make_pair(gml, H)
    lat, rel, sv = top.table()
    for i, s in enumerate(sv):
        ol, orl = orc.row(int(s), sv)
        assert np.array_equal(bits(lat[i]), bits(ol)), (name, i)
        assert np.array_equal(bits(rel[i]), bits(orl)), (name, i)


@pytest.mark.parametrize("name", ["complete30_ms", "complete25_dir", "sparse300_ms"])
def test_f64_lds_kernel_bit_exact(name, monkeypatch):
    """The f64 LDS kernel (SHD_SSSP_KERNEL=lds; the default for graphs of at
    most 4,096 vertices with fractional-ms latencies) forced on whole-ms
    graphs, where the integer-key LDS kernel is the default."""
    monkeypatch.setenv("SHD_SSSP_KERNEL", "lds")
    gml, H = GRAPHS[name]
    top, orc, _, _ = make_pair(gml, H)
    lat, rel, sv = top.table()
    for i, s in enumerate(sv):
        ol, orl = orc.row(int(s), sv)
        assert np.array_equal(bits(lat[i]), bits(ol)), (name, i)
        assert np.array_equal(bits(rel[i]), bits(orl)), (name, i)


@pytest.mark.parametrize("directed", [False, True])
def test_int_blocked_heap_deep_levels(directed):
    """Heaps of more than 8,191 nodes: the integer-key kernel's second level of
    HBM blocks (roots at level 13) and the crossings between block levels, on
    a dense whole-ms graph (V = 12,000, average degree 40), sampled rows
    against the oracle and every row against the f64 slab kernel."""
    import os
    gml = synth.sparse_graph_gml(12000, 0x5EED0072, avg_degree=40.0, directed=directed)
    top, orc, _, _ = make_pair(gml, 60)
    lat, rel, sv = top.table()
    for i in range(0, len(sv), max(1, len(sv) // 12)):
        ol, orl = orc.row(int(sv[i]), sv)
        assert np.array_equal(bits(lat[i]), bits(ol)), i
        assert np.array_equal(bits(rel[i]), bits(orl)), i
    os.environ["SHD_SSSP_KERNEL"] = "slab"
    try:
        top2, _, _, _ = make_pair(gml, 60)
        lat2, rel2, _ = top2.table()
    finally:
        del os.environ["SHD_SSSP_KERNEL"]
    assert np.array_equal(bits(lat), bits(lat2))
    assert np.array_equal(bits(rel), bits(rel2))


@pytest.mark.parametrize("waves", [1, 6])
def test_slab_kernel_persistent_rows(waves, monkeypatch):
    """Fewer slab waves than rows (SHD_SSSP_WAVES): each wave reuses its slab
    and LDS heap top for many sources; 6 waves = one partly idle block."""
    monkeypatch.setenv("SHD_SSSP_WAVES", str(waves))
    gml, H = GRAPHS["sparse5000_hbm"]
    top, orc, _, _ = make_pair(gml, H)
    lat, rel, sv = top.table()
    for i, s in enumerate(sv):
        ol, orl = orc.row(int(s), sv)
        assert np.array_equal(bits(lat[i]), bits(ol)), i
        assert np.array_equal(bits(rel[i]), bits(orl)), i


def test_reference_converter_fixture_graph():
    """The reference's own GML fixture (src/test/config/convert/
    topology.expected.gml, kept as data in tests/golden/): directed graph, one
    vertex, "50 ms" self-loop, loss 0."""
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "convert_topology_expected.gml")) as f:
        gml = f.read()
    top, orc, ips, _ = make_pair(gml, 3)
    for a in range(3):
        for b in range(3):
            assert top.get_latency(int(ips[a]), int(ips[b])) == 50.0
            assert top.get_reliability(int(ips[a]), int(ips[b])) == 1.0
            assert orc.latency(int(ips[a]), int(ips[b])) == 50.0


@pytest.mark.parametrize("directed", [False, True])
def test_direct_paths_bit_exact(directed):
    gml = synth.complete_graph_gml(20, 0x5EED0051, directed=directed)
    top, orc, _, _ = make_pair(gml, 60, use_sp=False)
    lat, rel, sv = top.table()
    for i, s in enumerate(sv):
        for j, d in enumerate(sv):
            ol, orl = orc.direct(int(s), int(d))
            assert bits(lat[i, j]) == bits(ol) and bits(rel[i, j]) == bits(orl)


@pytest.mark.parametrize("name,use_sp", [("complete30_ms", True), ("sparse300_ns", True),
                                         ("sparse200_dir_ns", True), ("complete25_dir", True),
                                         ("complete25_dir", False)])
def test_lookup_side_effects_match_reference(name, use_sp):
    """Random lookup sequences: values, the lazy touch/direction quirk and the
    running min that feeds worker_updateMinTimeJump."""
    gml, H = GRAPHS[name]
    top, orc, ips, _ = make_pair(gml, H, use_sp)
    rng = np.random.default_rng(7)
    for _ in range(600):
        a, b = (int(x) for x in rng.integers(0, H, 2))
        s, d = int(ips[a]), int(ips[b])
        assert bits(top.get_reliability(s, d)) == bits(orc.reliability(s, d))
        assert bits(top.get_latency(s, d)) == bits(orc.latency(s, d))
        assert top.is_routable(s, d) == orc.routable(s, d)
        assert bits(top.min_path_latency()) == bits(orc.min_path_latency())


def test_unattached_address():
    top, orc, ips, _ = make_pair(synth.complete_graph_gml(5, 3), 5)
    from shadow_amd import ShdError
    with pytest.raises(ShdError):
        top.get_latency(int(ips[0]), 0x01020304)
    assert orc.latency(int(ips[0]), 0x01020304) == -1
    assert top.is_routable(int(ips[0]), 0x01020304) is False


@pytest.fixture(params=["bucket", "rank", "slab", "slab_rankmajor", "slab_readlane", "slab_noagg", "rank_noagg",
                        "slab_unfused", "slab_wide", "part", "part_readlane", "part_lds", "part_s1", "part_s2", "part_s3", "part_s4",
                        "part_s3perm", "part_x5", "part_x6", "part_x7", "part_x8", "part_x9", "part_x7g3", "part_x8g5", "part_x9g7", "part_x10", "part_x11"])
def pipeline(request, monkeypatch):
    """The grouping pipelines of packet.hip (SHD_PACKET_PIPELINE: bucket,
    rank, slab, part -- the LDS-staged bucket partition + per-bucket LDS sort;
    the slab layout SHD_SLAB_LAYOUT, the segment sort's pass-1 key broadcast
    SHD_SEGSORT_LDS, the wave-aggregated destination slots SHD_DEST_AGG and
    the folded overflow placement SHD_ROUND_FUSE and the compact 16-B slab
    records SHD_SLAB_COMPACT, read per launch)."""
    monkeypatch.setenv("SHD_PACKET_PIPELINE", request.param.split("_")[0])
    monkeypatch.setenv("SHD_SLAB_LAYOUT", "rank" if request.param.endswith("rankmajor") else "host")
    monkeypatch.setenv("SHD_SEGSORT_LDS", "0" if request.param.endswith("readlane") else "1")
    monkeypatch.setenv("SHD_DEST_AGG", "0" if request.param.endswith("noagg") else "1")
    monkeypatch.setenv("SHD_ROUND_FUSE", "0" if request.param.endswith("unfused") else "1")
    monkeypatch.setenv("SHD_SLAB_COMPACT", "0" if request.param.endswith("wide") else "1")
    # part: the scatter's LDS-staged form and other instances (_xK), the
    # bucket sort's other instances (_sK), its in-order write (perm)
    p = request.param
    import re
    monkeypatch.setenv("SHD_PART_SCATTER", "0" if p.endswith("lds") else
                       re.match(r"\d+", p.split("_x")[1]).group(0) if "_x" in p else "1")
    # the pipelined scatter (_x7 / _x8) on a few workgroups (_gK): many
    # chunks per workgroup even on these small batches
    if "_x" in p and "g" in p.split("_x")[1]:
        monkeypatch.setenv("SHD_PART_PIPE_GRID", p.split("g")[-1])
    else:
        monkeypatch.delenv("SHD_PART_PIPE_GRID", raising=False)
    monkeypatch.setenv("SHD_PART_SORT", p.split("_s")[1][0] if "_s" in p else "0")
    monkeypatch.setenv("SHD_PART_PERM", "1" if p.endswith("perm") else "0")
    return p


ROUND_CASES = [
    # name, barrier, end_time, bootstrap_end, p_payload
    ("complete30_ms", 110_000_000, 10**15, 0, 0.9),
    ("complete40_ns", 110_000_000, 10**15, 0, 0.9),
    ("sparse300_ms", 110_000_000, 200_000_000, 0, 0.9),   # end-time drops
    ("sparse300_ns", 110_000_000, 10**15, 105_000_000, 0.5),  # bootstrap half the window
    ("sparse200_dir_ns", 110_000_000, 10**15, 0, 0.9),
    ("complete25_dir", 110_000_000, 10**15, 0, 1.0),
    ("1_gbit_switch", 110_000_000, 10**15, 0, 0.9),
]


@pytest.mark.parametrize("case", ROUND_CASES, ids=lambda c: c[0])
def test_packet_round_host_api_bit_exact(case, pipeline):
    name, barrier, end, boot, pp = case
    gml, H = GRAPHS[name]
    top, orc, ips, st = make_pair(gml, H)
    pk = synth.packet_batch(20000, H, 0x5EED0003, 100_000_000, 10_000_000, st, p_payload=pp)
    out, offs, status, mt = top.round(pk, barrier, end, boot)
    oout, ostatus, omt = orc.round(ips, pk, barrier, end, boot)
    assert np.array_equal(status, ostatus)
    assert mt == omt
    assert np.array_equal(out, oout)
    # segments: out[offs[h]:offs[h+1]] all go to h
    for h in range(H):
        assert (out["dst_host"][offs[h]:offs[h + 1]] == h).all()
    assert offs[-1] == len(out)
    # path packet counters (topology_incrementPathPacketCounter per kept packet,
    # counted on the device inside the round): single pairs, and every cached
    # path's count in the teardown log
    for a in range(0, H, max(1, H // 7)):
        for b in range(0, H, max(1, H // 5)):
            assert top.path_packet_count(int(ips[a]), int(ips[b])) == orc.packet_count(int(ips[a]), int(ips[b]))
    assert top.cached_paths_log() == orc.cached_paths_log()


def test_multi_round_state_carries():
    gml, H = GRAPHS["sparse300_ns"]
    top, orc, ips, st = make_pair(gml, H)
    states = st.copy()
    for r in range(3):
        pk = synth.packet_batch(5000, H, 0x5EED0100 + r, 100_000_000 * (r + 1), 10_000_000, states)
        out, _, status, mt = top.round(pk, 100_000_000 * (r + 1) + 10_000_000, 10**15)
        oout, ostatus, omt = orc.round(ips, pk, 100_000_000 * (r + 1) + 10_000_000, 10**15)
        assert np.array_equal(status, ostatus) and mt == omt and np.array_equal(out, oout)
        # advance each host's stream by the draws it made
        cnt = np.bincount(pk["src_host"], minlength=H)
        for h in range(H):
            for _ in range(cnt[h]):
                from shadow_amd.scenario import _rand_r
                _, states[h] = _rand_r(int(states[h]))
    assert bits(top.min_path_latency()) == bits(orc.min_path_latency())


def test_big_segments_bitonic_path(pipeline):
    """All packets to a few destinations: segments far above the LDS rank-sort
    size take the bitonic network."""
    gml, H = GRAPHS["complete30_ms"]
    top, orc, ips, st = make_pair(gml, H)
    pk = synth.packet_batch(12000, H, 0x5EED0200, 100_000_000, 10_000_000, st)
    pk["dst_host"] = np.where(pk["src_host"] % 3 == 0, 1, 2).astype(np.uint32)
    pk["dst_host"] = np.where(pk["dst_host"] == pk["src_host"], 0, pk["dst_host"]).astype(np.uint32)
    out, offs, status, mt = top.round(pk, 110_000_000, 10**15)
    oout, ostatus, omt = orc.round(ips, pk, 110_000_000, 10**15)
    assert np.array_equal(status, ostatus) and mt == omt and np.array_equal(out, oout)
    assert np.diff(offs).max() > 1024


def test_oversized_bucket_fallback(pipeline):
    """Skewed destinations: one partition bucket far above the LDS capacity of
    the per-bucket sort (16384 events) takes the in-place fallback."""
    gml, H = GRAPHS["complete30_ms"]
    top, orc, ips, st = make_pair(gml, H)
    pk = synth.packet_batch(60000, H, 0x5EED0210, 100_000_000, 10_000_000, st)
    hot = (pk["seq"] % 10) != 0  # 90 % of the packets go to host 1 (or 2 from host 1)
    pk["dst_host"] = np.where(hot, np.where(pk["src_host"] == 1, 2, 1), pk["dst_host"]).astype(np.uint32)
    out, offs, status, mt = top.round(pk, 110_000_000, 10**15)
    oout, ostatus, omt = orc.round(ips, pk, 110_000_000, 10**15)
    assert np.array_equal(status, ostatus) and mt == omt and np.array_equal(out, oout)
    assert offs[2] - offs[1] > 16384


@pytest.mark.parametrize("inst", ["default", "0", "1", "2", "3", "4"])
def test_part_sort_bucket_above_register_rows(inst, monkeypatch):
    """Buckets whose event count lies between a part-sort instance's register
    rows (kCap / kWG per thread, rounded down: 2,048 events for the 512-thread
    2,304-event instances) and the bucket cap: every event must still be
    loaded.  One destination per bucket (the batch's mean load of 1,900
    events per host sets shift 0 for the 2,304-event instances), destinations
    1..3 above 2,048 events."""
    monkeypatch.setenv("SHD_PACKET_PIPELINE", "part")
    if inst == "default":
        monkeypatch.delenv("SHD_PART_SORT", raising=False)
    else:
        monkeypatch.setenv("SHD_PART_SORT", inst)
    gml, H = GRAPHS["complete30_ms"]
    top, orc, ips, st = make_pair(gml, H)
    n = 1900 * H
    heavy = {1: 2300, 2: 2100, 3: 2049}
    rest = n - sum(heavy.values())
    others = [h for h in range(H) if h not in heavy]
    dst = np.concatenate([np.full(c, h, dtype=np.uint32) for h, c in heavy.items()] +
                         [np.array(others, dtype=np.uint32)[np.arange(rest) % len(others)]])
    rng = np.random.default_rng(0x5EED0220)
    dst = dst[rng.permutation(n)]
    src = rng.integers(0, H - 1, n).astype(np.uint32)
    src = np.where(src >= dst, src + 1, src).astype(np.uint32)
    pk = synth.packet_batch(n, H, 0x5EED0221, 100_000_000, 10_000_000, st, p_payload=0.0, pairs=(src, dst))
    out, offs, status, mt = top.round(pk, 110_000_000, 10**15)
    oout, ostatus, omt = orc.round(ips, pk, 110_000_000, 10**15)
    assert np.array_equal(status, ostatus) and mt == omt and np.array_equal(out, oout)
    assert np.diff(offs)[1] == 2300 and np.diff(offs)[3] == 2049


SEGMENT_EDGES = [16, 17, 63, 64, 65, 127, 128, 129, 255, 256, 257, 1023, 1024, 1025, 4095, 4096, 4097, 8192, 8193]


def test_segment_size_thresholds(pipeline):
    """Destination segments at every size threshold of the grouping kernels
    (one thread per event <= 16, wave ranks <= 64 / 128 / 256, the medium
    bitonic <= 1,024, the chunk sort's 4,096-event runs and the merge passes
    above), each side of it; the other hosts get a few events each."""
    gml, H = GRAPHS["complete30_ms"]
    top, orc, ips, st = make_pair(gml, H)
    loads = {h + 1: c for h, c in enumerate(SEGMENT_EDGES)}
    pk = _edge_batch(H, st, 0x5EED0230)
    out, offs, status, mt = top.round(pk, 110_000_000, 10**15)
    oout, ostatus, omt = orc.round(ips, pk, 110_000_000, 10**15)
    assert np.array_equal(status, ostatus) and mt == omt and np.array_equal(out, oout)
    assert [int(offs[h + 1] - offs[h]) for h in loads] == SEGMENT_EDGES


def _edge_batch(H, st, seed):
    """SEGMENT_EDGES events to hosts 1.., 5 to every other host, all kept."""
    loads = {h + 1: c for h, c in enumerate(SEGMENT_EDGES)}
    others = [h for h in range(H) if h not in loads]
    n = sum(loads.values()) + 5 * len(others)
    dst = np.concatenate([np.full(c, h, dtype=np.uint32) for h, c in loads.items()] +
                         [np.repeat(np.array(others, dtype=np.uint32), 5)])
    rng = np.random.default_rng(seed)
    dst = dst[rng.permutation(n)]
    src = rng.integers(0, H - 1, n).astype(np.uint32)
    src = np.where(src >= dst, src + 1, src).astype(np.uint32)
    return synth.packet_batch(n, H, seed + 1, 100_000_000, 10_000_000, st, p_payload=0.0, pairs=(src, dst))


@pytest.mark.parametrize("medium", ["auto", "0", "1"])
def test_sync_rounds_medium_segments_after_uniform(medium, monkeypatch):
    """Synchronous device rounds (null stream) on one workspace: a uniform
    round (no listed segment), then two with segments at every grouping
    threshold.  By default the second runs without k_segsort_medium (its
    predecessor listed nothing: k_segsort_mid sorts the medium segments) and
    the third with it again (SHD_MEDIUM_SEG=0 / 1: never / always)."""
    import torch
    monkeypatch.setenv("SHD_PACKET_PIPELINE", "part")
    monkeypatch.delenv("SHD_PART_SORT", raising=False)
    if medium == "auto":
        monkeypatch.delenv("SHD_MEDIUM_SEG", raising=False)
    else:
        monkeypatch.setenv("SHD_MEDIUM_SEG", medium)
    gml, H = GRAPHS["complete30_ms"]
    top, orc, ips, st = make_pair(gml, H)
    top.touch_all()
    lat, rel, sv = top.table()
    orc.preload(sv, lat, rel)
    batches = [synth.packet_batch(9000, H, 0x5EED0260, 100_000_000, 10_000_000, st, p_payload=0.0),
               _edge_batch(H, st, 0x5EED0262), _edge_batch(H, st, 0x5EED0264)]
    for pk in batches:
        n = len(pk)
        d_recs = torch.from_numpy(pk.view(np.uint8)).cuda()
        d_out = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
        d_off = torch.empty(H + 1, dtype=torch.int32, device="cuda")
        d_status = torch.empty(n, dtype=torch.uint8, device="cuda")
        d_cnt = torch.empty(2, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        top.process_device(d_recs.data_ptr(), n, 110_000_000, 10**15, 0, d_out.data_ptr(), d_off.data_ptr(),
                           d_status.data_ptr(), d_cnt.data_ptr(), 0)
        cnt = d_cnt.cpu().numpy().view(np.uint64)
        out = d_out.cpu().numpy().view(synth.DELIV_DTYPE)[:cnt[0]]
        oout, ostatus, omt = orc.round(ips, pk, 110_000_000, 10**15)
        assert np.array_equal(d_status.cpu().numpy(), ostatus) and cnt[1] == omt
        assert np.array_equal(out, oout)
        offs = d_off.cpu().numpy()
        assert np.array_equal(np.diff(offs), np.bincount(oout["dst_host"], minlength=H))


@pytest.mark.parametrize("per_dst", [40, 100, 200])
def test_packets_to_own_host(per_dst, pipeline):
    """A share of the packets addressed to their own host: no barrier clamp
    (host_single.c:187-192), so those deliveries land before the barrier and
    the segment's sort leaves its 31-bit barrier-relative keys for the 64-bit
    ones (and its time-bucket rank for the all-pairs one)."""
    gml, H = GRAPHS["sparse300_ms"]
    top, orc, ips, st = make_pair(gml, H)
    n = per_dst * H
    rng = np.random.default_rng(0x5EED0240 + per_dst)
    dst = rng.integers(0, H, n).astype(np.uint32)
    src = rng.integers(0, H, n).astype(np.uint32)
    own = rng.random(n) < 0.1
    src = np.where(own, dst, src).astype(np.uint32)
    pk = synth.packet_batch(n, H, 0x5EED0241 + per_dst, 100_000_000, 10_000_000, st, p_payload=0.5, pairs=(src, dst))
    out, offs, status, mt = top.round(pk, 110_000_000, 10**15)
    oout, ostatus, omt = orc.round(ips, pk, 110_000_000, 10**15)
    assert np.array_equal(status, ostatus) and mt == omt and np.array_equal(out, oout)
    assert (out["time"] < 110_000_000).any()


@pytest.mark.parametrize("ns", [False, True], ids=["ms", "ns"])
def test_long_path_latencies(ns, pipeline):
    """Path latencies up to 5 s (direct paths of a complete graph,
    use_shortest_path=false): deliveries 2^31 ns or more past the barrier
    leave the 16-B stage record and the 31-bit sort keys (wide events), and
    delays of 2^32 ns or more leave the 8-B packet-path table for the f64
    entry (kPtabFallback)."""
    gml = synth.complete_graph_gml(20, 0x5EED0250, ns_variant=ns, max_ms=5000)
    H = 60
    top, orc, ips, st = make_pair(gml, H, use_sp=False)
    pk = synth.packet_batch(30000, H, 0x5EED0251, 100_000_000, 10_000_000, st)
    out, offs, status, mt = top.round(pk, 110_000_000, 10**15)
    oout, ostatus, omt = orc.round(ips, pk, 110_000_000, 10**15)
    assert np.array_equal(status, ostatus) and mt == omt and np.array_equal(out, oout)
    late = out["time"] - 110_000_000
    assert (late >= 2**31).sum() > 1000 and (late >= 2**32).sum() > 500


def test_device_api_matches_oracle_after_touch_all(pipeline):
    import torch
    gml, H = GRAPHS["sparse300_ns"]
    top, orc, ips, st = make_pair(gml, H)
    top.touch_all()
    lat, rel, sv = top.table()
    orc.preload(sv, lat, rel)  # same rows released in slot order
    pk = synth.packet_batch(50000, H, 0x5EED0300, 100_000_000, 10_000_000, st)
    n = len(pk)
    d_recs = torch.from_numpy(pk.view(np.uint8)).cuda()
    d_out = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    d_off = torch.empty(H + 1, dtype=torch.int32, device="cuda")
    d_status = torch.empty(n, dtype=torch.uint8, device="cuda")
    d_cnt = torch.empty(2, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    top.process_device(d_recs.data_ptr(), n, 110_000_000, 10**15, 0, d_out.data_ptr(), d_off.data_ptr(),
                       d_status.data_ptr(), d_cnt.data_ptr(), 0)
    torch.cuda.synchronize()
    cnt = d_cnt.cpu().numpy().view(np.uint64)
    out = d_out.cpu().numpy().view(synth.DELIV_DTYPE)[:cnt[0]]
    oout, ostatus, omt = orc.round(ips, pk, 110_000_000, 10**15)
    assert np.array_equal(d_status.cpu().numpy(), ostatus)
    assert cnt[1] == omt
    assert np.array_equal(out, oout)
    # the device round counted every kept packet at its answering pair
    # (worker.c:551): every host pair's path count against the oracle's (the
    # device API applies no lookup side effect, so the oracle's round has
    # released self paths the product's has not: no log compare here)
    a, b = np.meshgrid(np.arange(H), np.arange(H), indexing="ij")
    count_check.check_against_oracle(top.path_packet_counts(), count_check.slot_map(top.verts), orc, ips,
                                     a.ravel(), b.ravel())


@pytest.mark.parametrize("mode", ["log", "log_small", "atomic", "oom", "oom64_small"])
@pytest.mark.parametrize("api", ["host", "device"])
def test_path_counters_spill_to_host(api, mode, monkeypatch):
    """The device counters move to the host map before any could wrap
    (SHD_PCNT_SPILL_AT lowers the 2^31 threshold to 3): five rounds, every
    cached path's count equal to the oracle's after each.  Modes: the log
    (folded at each read), a log of 4,000 records (each round but the first
    folds the previous one first: SHD_PCNT_LOG) and the per-packet atomic.
    oom: the dense counters' allocation fails (SHD_DEBUG_PCNT_OOM), so the
    rounds only log and the log drains into the host map -- with u32 keys,
    and with u64 keys (the form of tables of 2^32 entries or more) in a log
    of 4,000 records that drains before each round."""
    import torch
    monkeypatch.setenv("SHD_PCNT_SPILL_AT", "3")
    monkeypatch.setenv("SHD_PCNT", "atomic" if mode == "atomic" else "log")
    if mode.endswith("_small"):
        monkeypatch.setenv("SHD_PCNT_LOG", "4000")
    if mode.startswith("oom"):
        monkeypatch.setenv("SHD_DEBUG_PCNT_OOM", "64" if "64" in mode else "1")
    gml, H = GRAPHS["complete30_ms"]
    top, orc, ips, st = make_pair(gml, H)
    if api == "device":
        top.touch_all()
        lat, rel, sv = top.table()
        orc.preload(sv, lat, rel)
    for r in range(5):
        pk = synth.packet_batch(3000, H, 0x5EED0310 + r, 100_000_000, 10_000_000, st)
        if api == "host":
            top.round(pk, 110_000_000, 10**15)
        else:
            n = len(pk)
            d_recs = torch.from_numpy(pk.view(np.uint8)).cuda()
            d_out = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
            d_off = torch.empty(H + 1, dtype=torch.int32, device="cuda")
            d_status = torch.empty(n, dtype=torch.uint8, device="cuda")
            d_cnt = torch.empty(2, dtype=torch.int64, device="cuda")
            torch.cuda.synchronize()
            top.process_device(d_recs.data_ptr(), n, 110_000_000, 10**15, 0, d_out.data_ptr(), d_off.data_ptr(),
                               d_status.data_ptr(), d_cnt.data_ptr(), 0)
        orc.round(ips, pk, 110_000_000, 10**15)
        if api == "host":
            assert top.cached_paths_log() == orc.cached_paths_log(), f"round {r}"
        else:
            a, b = np.meshgrid(np.arange(H), np.arange(H), indexing="ij")
            count_check.check_against_oracle(top.path_packet_counts(), count_check.slot_map(top.verts), orc, ips,
                                             a.ravel(), b.ravel())
    assert max(int(x.split("PacketCount=")[1].split()[0]) for x in orc.cached_paths_log()) > 3  # spilled


@pytest.mark.parametrize("fold", ["d8", "u32", "mixed"])
@pytest.mark.parametrize("log", ["250000", "-"])
def test_path_counter_fold_multi_region(log, fold, monkeypatch):
    """The counter log's fold over several coarse buckets and hundreds of
    32K-counter regions (A ~ 5,600 slots: 31M counters), three device rounds
    of 200k packets: every counter against the numpy restatement after each
    round.  SHD_PCNT_LOG=250000 makes the second and third round fold the
    logs before them first; "-" folds only at each read.  fold: into the u8
    delta layer (default; two hot pairs take 200 / 5,000 / 200 and 200 /
    200 / 200 counts, so bytes pass 255 within one fold and across folds and
    move into the u32 counters), into the u32 counters alone (SHD_FOLD_D8=0),
    or alternating per round (both layers hold counts)."""
    import torch
    if log != "-":
        monkeypatch.setenv("SHD_PCNT_LOG", log)
    monkeypatch.setenv("SHD_PCNT", "log")
    gml = synth.sparse_graph_gml(7000, 0x5EED0F11)
    H = 14_000
    top = Topology(gml)
    ips, st, verts = scenario.register_hosts(top, H, seed=1)
    A = top.slot_count()
    assert A * A > (1 << 24)  # several coarse buckets (2^22 counters each)
    top.touch_all()
    hslot = count_check.slot_map(verts)
    want = np.zeros((A, A), dtype=np.uint64)
    n = 200_000
    for r in range(3):
        pk = synth.packet_batch(n, H, 0x5EED0F12 + r, 100_000_000, 10_000_000, st)
        # hot pairs: many counts on one counter
        k = 5000 if r == 1 else 200
        pk["src_host"][:k], pk["dst_host"][:k] = 3, 7
        pk["src_host"][k:k + 200], pk["dst_host"][k:k + 200] = 5, 9
        if fold == "u32" or (fold == "mixed" and r == 1):
            monkeypatch.setenv("SHD_FOLD_D8", "0")
        else:
            monkeypatch.delenv("SHD_FOLD_D8", raising=False)
        d_recs = torch.from_numpy(pk.view(np.uint8)).cuda()
        d_out = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
        d_off = torch.empty(H + 1, dtype=torch.int32, device="cuda")
        d_status = torch.empty(n, dtype=torch.uint8, device="cuda")
        d_cnt = torch.empty(2, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        top.process_device(d_recs.data_ptr(), n, 110_000_000, 10**15, 0, d_out.data_ptr(), d_off.data_ptr(),
                           d_status.data_ptr(), d_cnt.data_ptr(), 0)
        torch.cuda.synchronize()
        want += count_check.expected_counts(hslot, pk, d_status.cpu().numpy(), A)
        got = top.path_packet_counts()
        bad = np.argwhere(got != want)
        assert len(bad) == 0, f"round {r}: {len(bad)} counters differ, first {bad[:4].tolist()}"


@pytest.mark.parametrize("hot_every", [4, 6])
@pytest.mark.parametrize("rounds_per_fold", [1, 2])
def test_path_counter_fold_hot_region(rounds_per_fold, hot_every, monkeypatch):
    """A hot sender (Zipf-like: 450k of 600k packets from one host to uniform
    destinations -- every packet but each hot_every-th) puts more than the
    add's chunk (2^18 keys) into one 32K counter region: the fold splits that
    region over several workgroups that add with device atomics.  hot_every
    6, folded each round: the 100k packets of every sixth one go to the hot
    sender's region alone with the rest uniform (a big region of one chunk:
    more keys than the u16 LDS counters of the small regions hold, less than
    a chunk).  Every counter against the numpy restatement, folded after each
    round or after two."""
    import torch
    monkeypatch.setenv("SHD_PCNT", "log")
    gml = synth.sparse_graph_gml(3000, 0x5EED0F21)
    H = 6_000
    top = Topology(gml)
    ips, st, verts = scenario.register_hosts(top, H, seed=1)
    A = top.slot_count()
    top.touch_all()
    hslot = count_check.slot_map(verts)
    hot = int(np.argmin(hslot))  # (slot 0: its row owns its pairs with every later slot)
    want = np.zeros((A, A), dtype=np.uint64)
    n = 600_000
    for r in range(2):
        pk = synth.packet_batch(n, H, 0x5EED0F22 + r, 100_000_000, 10_000_000, st)
        src = (np.where(np.arange(n) % 4 != 0, hot, pk["src_host"]) if hot_every == 4 else
               np.where(np.arange(n) % 6 == 0, hot, pk["src_host"])).astype(np.uint32)
        dst = synth.redraw_destinations(pk, H, 0x5EED0F30 + r)["dst_host"]
        dst = np.where(dst == src, (src + 1) % H, dst).astype(np.uint32)
        pk = synth.packet_batch(n, H, 0x5EED0F22 + r, 100_000_000, 10_000_000, st, pairs=(src, dst))
        d_recs = torch.from_numpy(pk.view(np.uint8)).cuda()
        d_out = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
        d_off = torch.empty(H + 1, dtype=torch.int32, device="cuda")
        d_status = torch.empty(n, dtype=torch.uint8, device="cuda")
        d_cnt = torch.empty(2, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        top.process_device(d_recs.data_ptr(), n, 110_000_000, 10**15, 0, d_out.data_ptr(), d_off.data_ptr(),
                           d_status.data_ptr(), d_cnt.data_ptr(), 0)
        torch.cuda.synchronize()
        want += count_check.expected_counts(hslot, pk, d_status.cpu().numpy(), A)
        if (r + 1) % rounds_per_fold == 0:
            got = top.path_packet_counts()
            bad = np.argwhere(got != want)
            assert len(bad) == 0, f"round {r}: {len(bad)} counters differ, first {bad[:4].tolist()}"
    assert want.max() > 0 and int((want > 0).sum(axis=1).max()) > 1000


def test_deliv_sort_device_against_lexsort(pipeline):
    import torch
    top, _, _, _ = make_pair(synth.complete_graph_gml(5, 3), 5)
    rng = np.random.default_rng(3)
    n, lo, hi = 200000, 1000, 3000
    ev = np.zeros(n, dtype=synth.DELIV_DTYPE)
    ev["time"] = rng.integers(0, 50, n)
    ev["dst_host"] = rng.integers(lo, hi, n)
    ev["src_host"] = rng.integers(0, 5000, n)
    ev["seq"] = np.arange(n) * 7 % 100003 + rng.integers(0, 3, n) * 1000000
    ev["pkt_index"] = np.arange(n)
    ev["dst_host"][:5000] = lo + 7  # one big segment
    d_in = torch.from_numpy(ev.view(np.uint8)).cuda()
    d_out = torch.empty_like(d_in)
    d_off = torch.empty(hi - lo + 1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    top.deliv_sort_device(d_in.data_ptr(), n, lo, hi, d_out.data_ptr(), d_off.data_ptr(), 0)
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().view(synth.DELIV_DTYPE)
    order = np.lexsort((ev["pkt_index"], ev["seq"], ev["src_host"], ev["time"], ev["dst_host"]))
    want = ev[order]
    # (time, src, seq) ties are broken arbitrarily by construction here; compare keys
    for k in ("dst_host", "time", "src_host", "seq"):
        assert np.array_equal(got[k], want[k]), k
    offs = d_off.cpu().numpy()
    assert offs[-1] == n and np.array_equal(np.diff(offs), np.bincount(ev["dst_host"] - lo, minlength=hi - lo))


def test_deliv_sort_skewed_destinations_merge_passes(pipeline):
    """Skewed destinations (a popular server): segments of 150k, 40k, 9k, 5k,
    4097 and 4096 events -- 6, 4, 2, 1, 1 and 0 merge passes over the
    4096-event LDS runs -- beside thousands of small ones; every event must
    come out in event_compare order (the keys are distinct: exact compare)."""
    import torch
    top, _, _, _ = make_pair(synth.complete_graph_gml(5, 3), 5)
    rng = np.random.default_rng(11)
    lo, hi = 500, 4500
    sizes = [150_000, 40_000, 9_000, 5_000, 4_097, 4_096]
    hot = np.concatenate([np.full(k, lo + 3 * i, dtype=np.int64) for i, k in enumerate(sizes)])
    rest = rng.integers(lo, hi, 100_000)
    dst = np.concatenate([hot, rest])
    n = len(dst)
    ev = np.zeros(n, dtype=synth.DELIV_DTYPE)
    ev["dst_host"] = rng.permutation(dst)
    ev["time"] = 110_000_000 + rng.integers(0, 2_000, n) * 1_000  # many equal times
    ev["src_host"] = rng.integers(0, 300, n)                       # many equal (time, src)
    ev["seq"] = rng.permutation(n)                                 # distinct: a total order
    ev["pkt_index"] = np.arange(n)
    d_in = torch.from_numpy(ev.view(np.uint8)).cuda()
    d_out = torch.empty_like(d_in)
    d_off = torch.empty(hi - lo + 1, dtype=torch.int32, device="cuda")
    for _ in range(2):  # the second call reuses the workspace and its merge metadata
        top.deliv_sort_device(d_in.data_ptr(), n, lo, hi, d_out.data_ptr(), d_off.data_ptr(), 0)
        torch.cuda.synchronize()
        got = d_out.cpu().numpy().view(synth.DELIV_DTYPE)
        want = ev[np.lexsort((ev["seq"], ev["src_host"], ev["time"], ev["dst_host"]))]
        assert np.array_equal(got, want)
        offs = d_off.cpu().numpy()
        assert np.array_equal(np.diff(offs), np.bincount(ev["dst_host"] - lo, minlength=hi - lo))


def test_multi_gpu_row_shards_assemble():
    """Rows built in shards into a caller-owned (torch) table == one-shot build."""
    import torch
    gml, H = GRAPHS["sparse300_ns"]
    top, _, _, _ = make_pair(gml, H)
    lat, rel, sv = top.table()
    top2 = Topology(gml)
    scenario.register_hosts(top2, H, 1)
    A = top2.slot_count()
    tab = torch.empty(A * A * 2, dtype=torch.float64, device="cuda")
    for lo in range(0, A, 97):
        top2.build_rows_device(lo, min(A, lo + 97), tab.data_ptr())
    torch.cuda.synchronize()
    top2.adopt_table_device(tab.data_ptr())
    lat2, rel2, _ = top2.table()
    assert np.array_equal(bits(lat), bits(lat2)) and np.array_equal(bits(rel), bits(rel2))


def test_full_size_c3_round_bit_exact():
    """BASELINE configs[3] at full size: 10M packets over 100k hosts on the
    V=20k sparse graph (the whole 19,870 x 19,870 table resident), device API.
    Senders and receivers are the hosts attached to the first 1,000 table
    slots so that the oracle's preloaded rows stay small; every packet still
    goes through the full-size kernels, host map and partition geometry."""
    import torch
    H, V = 100_000, 20_000
    gml = synth.sparse_graph_gml(V, 0x5EED0002)
    top = Topology(gml)
    ips, st, verts = scenario.register_hosts(top, H, seed=1)
    A = top.slot_count()
    sv = np.unique(verts).astype(np.int32)  # slots = attached vertices, ascending
    assert len(sv) == A
    full = torch.empty(A * A * 2, dtype=torch.float64, device="cuda")
    top.build_rows_device(0, A, full.data_ptr())
    torch.cuda.synchronize()
    top.adopt_table_device(full.data_ptr())
    top.touch_all()
    k = 1000
    blk = full.view(A, A, 2)[:k, :k].cpu().numpy()
    orc = O.OracleTopology(gml)
    ips_o, st_o, verts_o = scenario.register_hosts(orc, H, seed=1)
    assert (verts == verts_o).all()
    for i in (0, 1, A // 2, A - 1):  # full-length rows of the slab kernel vs the oracle's Dijkstra
        ol, orl = orc.row(int(sv[i]), sv)
        row = full.view(A, A, 2)[i].cpu().numpy()
        assert np.array_equal(bits(row[:, 0]), bits(ol)) and np.array_equal(bits(row[:, 1]), bits(orl)), i
    orc.preload(sv[:k], np.ascontiguousarray(blk[:, :, 0]), np.ascontiguousarray(blk[:, :, 1]))
    hosts = np.flatnonzero(np.isin(verts, sv[:k])).astype(np.uint32)
    n = 10_000_000
    pk = synth.packet_batch(n, H, 0x5EED0400, 100_000_000, 10_000_000, st, hosts=hosts)
    d_recs = torch.from_numpy(pk.view(np.uint8)).cuda()
    d_out = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    d_off = torch.empty(H + 1, dtype=torch.int32, device="cuda")
    d_status = torch.empty(n, dtype=torch.uint8, device="cuda")
    d_cnt = torch.empty(2, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    top.process_device(d_recs.data_ptr(), n, 110_000_000, 10**15, 0, d_out.data_ptr(), d_off.data_ptr(),
                       d_status.data_ptr(), d_cnt.data_ptr(), 0)
    torch.cuda.synchronize()
    cnt = d_cnt.cpu().numpy().view(np.uint64)
    out = d_out.cpu().numpy().view(synth.DELIV_DTYPE)[:cnt[0]]
    oout, ostatus, omt = orc.round(ips_o, pk, 110_000_000, 10**15)
    assert np.array_equal(d_status.cpu().numpy(), ostatus)
    assert cnt[1] == omt
    assert np.array_equal(out, oout)
    offs = d_off.cpu().numpy().astype(np.int64)
    assert offs[-1] == len(out) and np.array_equal(np.diff(offs), np.bincount(out["dst_host"], minlength=H))


# ---- edge cases of the hand-off (empty / single / all dropped / bad ids) ----

def test_empty_and_single_packet_rounds(pipeline):
    gml, H = GRAPHS["complete30_ms"]
    top, orc, ips, st = make_pair(gml, H)
    pk = synth.packet_batch(1, H, 0x5EED0400, 100_000_000, 10_000_000, st)
    for batch in (pk[:0], pk):
        out, offs, status, mt = top.round(batch, 110_000_000, 10**15)
        oout, ostatus, omt = orc.round(ips, batch, 110_000_000, 10**15)
        assert len(status) == len(batch)
        assert np.array_equal(status, ostatus) and mt == omt and np.array_equal(out, oout)
        assert offs[-1] == len(out)
    assert mt != 2**64 - 1  # the single packet was delivered


def test_every_packet_dropped(pipeline):
    """Loss 1.0 on every edge (reliability 0): only draws of exactly 0 keep a
    packet with payload; then an end time before the window drops the rest."""
    import re
    gml = re.sub(r"packet_loss [0-9.eE+-]+", "packet_loss 1.0", synth.complete_graph_gml(20, 0x5EED0071))
    top, orc, ips, st = make_pair(gml, 60)
    pk = synth.packet_batch(30000, 60, 0x5EED0410, 100_000_000, 10_000_000, st, p_payload=1.0)
    out, offs, status, mt = top.round(pk, 110_000_000, 10**15)
    oout, ostatus, omt = orc.round(ips, pk, 110_000_000, 10**15)
    assert np.array_equal(status, ostatus) and mt == omt and np.array_equal(out, oout)
    DELIVERED, LOSS = 1, 0  # shdnet.h: SHD_DROPPED_LOSS = 0, SHD_DELIVERED = 1, SHD_DROPPED_END = 2
    assert len(out) == (status == DELIVERED).sum() < 10 and (status == LOSS).sum() >= len(pk) - 10
    top2, orc2, ips2, st2 = make_pair(GRAPHS["complete30_ms"][0], 90)
    pk2 = synth.packet_batch(30000, 90, 0x5EED0411, 100_000_000, 10_000_000, st2, p_payload=0.5)
    out, offs, status, mt = top2.round(pk2, 110_000_000, 100_000_000)  # end time = window start
    oout, ostatus, omt = orc2.round(ips2, pk2, 110_000_000, 100_000_000)
    assert np.array_equal(status, ostatus) and mt == omt == 2**64 - 1 and len(out) == len(oout) == 0
    assert offs[-1] == 0


def test_compact_slab_fallbacks(pipeline):
    """Events the 16-B compact slab record cannot hold go whole to the 32-B
    slab (packet.hip CSlab): srcHostEventIDs of 2^32 and more, and self
    deliveries more than 2^31 ns before the barrier; mixed with compact ones
    in the same destination segments, and rounds far from time 0."""
    gml, H = GRAPHS["complete30_ms"]
    top, orc, ips, st = make_pair(gml, H)
    barrier = 10_000_000_000
    pk = synth.packet_batch(40000, H, 0x5EED0420, barrier - 10_000_000, 10_000_000, st)
    rng = np.random.default_rng(0x5EED0421)
    big = rng.random(len(pk)) < 0.1
    pk["seq"][big] += np.uint64(1 << 32)  # (src, seq) stays unique: a total order
    early = np.flatnonzero(rng.random(len(pk)) < 0.05)
    pk["dst_host"][early] = pk["src_host"][early]
    pk["now"][early] = barrier - 3_000_000_000  # self delivery ~3 s before the barrier: no clamp
    out, offs, status, mt = top.round(pk, barrier, 10**15)
    oout, ostatus, omt = orc.round(ips, pk, barrier, 10**15)
    assert np.array_equal(status, ostatus) and mt == omt and np.array_equal(out, oout)
    assert (out["seq"] >= 1 << 32).sum() > 1000 and (out["time"] < barrier - 2**31).sum() > 100


def test_all_events_wide(pipeline):
    """Every event outside the compact forms (srcHostEventIDs of 2^32 and
    more: a host's event counter in a long simulation), so every bucket of
    the part pipeline has wide events: each reads only its own from the
    bucket-grouped wide list (k_wide_group); outputs equal the oracle's."""
    gml, H = GRAPHS["sparse300_ms"]
    top, orc, ips, st = make_pair(gml, H)
    pk = synth.packet_batch(120000, H, 0x5EED0430, 100_000_000, 10_000_000, st)
    pk["seq"] += np.uint64(3 << 32)
    out, offs, status, mt = top.round(pk, 110_000_000, 10**15)
    oout, ostatus, omt = orc.round(ips, pk, 110_000_000, 10**15)
    assert np.array_equal(status, ostatus) and mt == omt and np.array_equal(out, oout)
    assert len(out) > 100000


def test_device_api_unknown_hosts_not_delivered(pipeline):
    """Records naming host ids outside the registered range get status 0xff and
    no event; every other record is decided exactly as the oracle does."""
    import torch
    gml, H = GRAPHS["sparse300_ns"]
    top, orc, ips, st = make_pair(gml, H)
    top.touch_all()
    lat, rel, sv = top.table()
    orc.preload(sv, lat, rel)
    pk = synth.packet_batch(20000, H, 0x5EED0420, 100_000_000, 10_000_000, st)
    bad = np.zeros(len(pk), dtype=bool)
    bad[::97] = True
    pk["dst_host"][::194] = H + 5
    pk["src_host"][97::194] = 0xFFFFFFF0
    n = len(pk)
    d_recs = torch.from_numpy(pk.view(np.uint8)).cuda()
    d_out = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    d_off = torch.empty(H + 1, dtype=torch.int32, device="cuda")
    d_status = torch.empty(n, dtype=torch.uint8, device="cuda")
    d_cnt = torch.empty(2, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    top.process_device(d_recs.data_ptr(), n, 110_000_000, 10**15, 0, d_out.data_ptr(), d_off.data_ptr(),
                       d_status.data_ptr(), d_cnt.data_ptr(), 0)
    torch.cuda.synchronize()
    status = d_status.cpu().numpy()
    cnt = d_cnt.cpu().numpy().view(np.uint64)
    out = d_out.cpu().numpy().view(synth.DELIV_DTYPE)[:cnt[0]].copy()
    assert (status[bad] == 0xFF).all()
    good = np.flatnonzero(~bad)
    oout, ostatus, omt = orc.round(ips, pk[good], 110_000_000, 10**15)
    oout = oout.copy()
    oout["pkt_index"] = good[oout["pkt_index"]]
    assert np.array_equal(status[good], ostatus) and cnt[1] == omt
    assert np.array_equal(out, oout)


@pytest.mark.parametrize("name", ["sparse300_ns", "sparse200_dir_ns", "sparse5000_hbm"])
def test_device_resident_table_matches_mirrored(name, pipeline):
    """adopt_table_device_resident (no host mirror) + touch_all ==
    adopt_table_device + touch_all: same released minimum (touch_all's rows
    released by the device pass in slot order), same host lookups
    (single-entry device reads), same device round as the oracle."""
    import torch
    from shadow_amd import ShdError
    gml, H = GRAPHS[name]
    top, orc, ips, st = make_pair(gml, H)
    top.touch_all()
    lat, rel, sv = top.table()
    orc.preload(sv, lat, rel)
    top2 = Topology(gml)
    scenario.register_hosts(top2, H, 1)
    A = top2.slot_count()
    tab = torch.empty(A * A * 2, dtype=torch.float64, device="cuda")
    top2.build_rows_device(0, A, tab.data_ptr())
    torch.cuda.synchronize()
    top2.adopt_table_device_resident(tab.data_ptr())
    assert top2.min_path_latency() == 0  # lazy: nothing released at adoption
    top2.touch_all()
    assert bits(top2.min_path_latency()) == bits(top.min_path_latency())
    with pytest.raises(ShdError):
        top2.adopt_table_device_resident(tab.data_ptr())  # rows already released: -EBUSY
    for a in range(0, H, max(1, H // 9)):
        for b in range(0, H, max(1, H // 7)):
            s, d = int(ips[a]), int(ips[b])
            assert bits(top2.get_latency(s, d)) == bits(top.get_latency(s, d))
            assert bits(top2.get_reliability(s, d)) == bits(top.get_reliability(s, d))
    pk = synth.packet_batch(30000, H, 0x5EED0430, 100_000_000, 10_000_000, st)
    n = len(pk)
    d_recs = torch.from_numpy(pk.view(np.uint8)).cuda()
    d_out = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    d_off = torch.empty(H + 1, dtype=torch.int32, device="cuda")
    d_status = torch.empty(n, dtype=torch.uint8, device="cuda")
    d_cnt = torch.empty(2, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    top2.process_device(d_recs.data_ptr(), n, 110_000_000, 10**15, 0, d_out.data_ptr(), d_off.data_ptr(),
                        d_status.data_ptr(), d_cnt.data_ptr(), 0)
    torch.cuda.synchronize()
    cnt = d_cnt.cpu().numpy().view(np.uint64)
    out = d_out.cpu().numpy().view(synth.DELIV_DTYPE)[:cnt[0]]
    oout, ostatus, omt = orc.round(ips, pk, 110_000_000, 10**15)
    assert np.array_equal(d_status.cpu().numpy(), ostatus) and cnt[1] == omt
    assert np.array_equal(out, oout)


def test_device_resident_needs_shortest_path():
    import torch
    from shadow_amd import ShdError
    gml, H = GRAPHS["complete30_ms"]
    top = Topology(gml, use_shortest_path=False)
    scenario.register_hosts(top, H, 1)
    A = top.slot_count()
    tab = torch.empty(A * A * 2, dtype=torch.float64, device="cuda")
    top.build_rows_device(0, A, tab.data_ptr())
    torch.cuda.synchronize()
    with pytest.raises(ShdError):
        top.adopt_table_device_resident(tab.data_ptr())


def test_packet_round_zipf_senders(pipeline):
    """C3's Zipf variant: skewed senders, so a few hosts send
    most packets (long rand_r advances, many equal-time ties per sender)."""
    gml, H = GRAPHS["sparse300_ms"]
    top, orc, ips, st = make_pair(gml, H)
    pk = synth.packet_batch(50000, H, 0x5EED0440, 100_000_000, 10_000_000, st, zipf=True)
    assert np.bincount(pk["src_host"], minlength=H).max() > 20 * len(pk) / H  # skewed
    out, offs, status, mt = top.round(pk, 110_000_000, 10**15)
    oout, ostatus, omt = orc.round(ips, pk, 110_000_000, 10**15)
    assert np.array_equal(status, ostatus) and mt == omt and np.array_equal(out, oout)
    assert offs[-1] == len(out)


def test_medium_segments_lds_path(pipeline):
    """Destinations with 257..4096 events in a round (a server host receiving
    from many clients): the LDS bitonic segment sort."""
    gml, H = GRAPHS["complete30_ms"]
    top, orc, ips, st = make_pair(gml, H)
    pk = synth.packet_batch(14000, H, 0x5EED0450, 100_000_000, 10_000_000, st)
    hot = (pk["seq"] % 4) != 0  # 3/4 of the packets go to hosts 1..8
    d = (1 + (pk["seq"] * 7 + pk["src_host"]) % 8).astype(np.uint32)
    d = np.where(d == pk["src_host"], 9, d).astype(np.uint32)
    pk["dst_host"] = np.where(hot, d, pk["dst_host"]).astype(np.uint32)
    out, offs, status, mt = top.round(pk, 110_000_000, 10**15)
    oout, ostatus, omt = orc.round(ips, pk, 110_000_000, 10**15)
    assert np.array_equal(status, ostatus) and mt == omt and np.array_equal(out, oout)
    seg = np.diff(offs)
    assert ((seg > 256) & (seg <= 4096)).sum() >= 4


@pytest.mark.parametrize("name", ["sparse200_dir_ns", "complete25_dir"])
def test_send_time_append_interleaved_with_lookups(name):
    """Within one round, worker sends (shd_round_append_worker, whose lookup
    side effect happens at send time like topology_getReliability at
    worker.c:539) interleave with other callers' lookups (topology_isRoutable
    at socket.c:808, worker_getLatency at tcp.c:392-393).  On a directed
    ns-resolution graph the owner of a pair -- and with it the bits of every
    later answer and the min-jump sequence -- depends on that order.  The
    oracle replays the same serial sequence; values, the callback sequence
    and the round's output must match."""
    gml, H = GRAPHS[name]
    top, orc, ips, st = make_pair(gml, H)
    top.record_min_jump()
    check = __import__("shadow_amd._lib", fromlist=["check"]).check
    lib = __import__("shadow_amd._lib", fromlist=["lib"]).lib()
    check(lib.shd_round_set_workers(top.handle, 3))
    check(lib.shd_round_begin(top.handle, 110_000_000, 10**15, 0))
    pk = synth.packet_batch(3000, H, 0x5EED0500, 100_000_000, 10_000_000, st)
    rng = np.random.default_rng(11)
    order = []  # (worker, record) in append order; pkt_index counts worker 0's first
    for i in range(len(pk)):
        for _ in range(int(rng.integers(0, 3))):  # lookups by other callers between two sends
            a, b = (int(x) for x in rng.integers(0, H, 2))
            s, d = int(ips[a]), int(ips[b])
            if rng.integers(0, 2):
                assert top.is_routable(s, d) == orc.routable(s, d)
            else:
                assert bits(top.get_latency(s, d)) == bits(orc.latency(s, d))
        w = int(rng.integers(0, 3))
        rec = pk[i:i + 1]
        check(lib.shd_round_append_worker(top.handle, w, rec.ctypes.data, 1))
        orc.reliability(int(ips[rec["src_host"][0]]), int(ips[rec["dst_host"][0]]))  # the send's lookup
        order.append((w, i))
        assert bits(top.min_path_latency()) == bits(orc.min_path_latency())
        # the callback fires once per decreasing row release; the reference
        # fires per stored entry in its target iteration order, ending at the
        # same value (controller_updateMinTimeJump keeps the last, :141-153)
        assert (not top.min_jump_calls and orc.min_jump_updates() == 0) or \
            bits(top.min_jump_calls[-1]) == bits(orc.min_path_latency())
        assert len(top.min_jump_calls) <= orc.min_jump_updates()
        assert top.next_min_jump_ns() == orc.next_min_jump_ns()
    # collect: records in worker order, each worker's in append order
    perm = [i for w in range(3) for (ww, i) in order if ww == w]
    staged = pk[perm]
    out = np.zeros(len(pk), dtype=synth.DELIV_DTYPE)
    offs = np.zeros(H + 1, dtype=np.uint32)
    status = np.zeros(len(pk), dtype=np.uint8)
    nout, mt = C.c_size_t(), C.c_uint64()
    check(lib.shd_round_collect(top.handle, out.ctypes.data, len(out), C.byref(nout), offs.ctypes.data,
                                status.ctypes.data, C.byref(mt)))
    oout, ostatus, omt = orc.round(ips, staged, 110_000_000, 10**15)  # lookups are hits now: no side effects
    assert np.array_equal(status, ostatus) and mt.value == omt
    assert np.array_equal(out[:nout.value], oout)
    assert top.min_jump_calls == sorted(set(top.min_jump_calls), reverse=True)  # strictly decreasing


@pytest.mark.parametrize("resident", [False, True])
def test_lookup_batch_matches_single_lookups(resident):
    """shd_topology_lookup_batch: the same answers and side effects as one
    topology_getLatency call per pair, in order; on a device-resident table
    they come from one device gather (no per-lookup PCIe read)."""
    import torch
    gml, H = GRAPHS["sparse200_dir_ns"]
    top, orc, ips, _ = make_pair(gml, H)
    rng = np.random.default_rng(21)
    a, b = rng.integers(0, H, 3000), rng.integers(0, H, 3000)
    s, d = ips[a], ips[b]
    if resident:
        A = top.slot_count()
        tab = torch.empty(A * A * 2, dtype=torch.float64, device="cuda")
        top.build_rows_device(0, A, tab.data_ptr())
        torch.cuda.synchronize()
        top.adopt_table_device_resident(tab.data_ptr())  # lazy: the batch's touches release rows on the device
    top.record_min_jump()
    lat, rel = top.lookup_batch(s, d)
    for i in range(len(s)):
        assert bits(lat[i]) == bits(orc.latency(int(s[i]), int(d[i])))
        assert bits(rel[i]) == bits(orc.reliability(int(s[i]), int(d[i])))
    assert bits(top.min_path_latency()) == bits(orc.min_path_latency())
    assert top.next_min_jump_ns() == orc.next_min_jump_ns()
    assert top.cached_paths_log() == orc.cached_paths_log()  # the same pairs from the same rows


@pytest.mark.parametrize("name,use_sp", [("1_gbit_switch", True), ("complete30_ms", True), ("sparse300_ns", True),
                                         ("sparse200_dir_ns", True), ("complete25_dir", False),
                                         ("sparse5000_hbm", True)])
def test_teardown_path_log_matches_reference(name, use_sp):
    """topology_free's cached-path log after random lookups and counted
    packets: the same lines (ids, indices, %f latency / reliability, packet
    counts, isDirect) as the oracle's literal cache."""
    gml, H = GRAPHS[name]
    top, orc, ips, _ = make_pair(gml, H, use_sp)
    rng = np.random.default_rng(11)
    for _ in range(400):
        a, b = (int(x) for x in rng.integers(0, H, 2))
        s, d = int(ips[a]), int(ips[b])
        assert bits(top.get_latency(s, d)) == bits(orc.latency(s, d))
        if rng.random() < 0.5:
            top.increment_path_packet_counter(s, d)
            orc.increment(s, d)
    got = top.cached_paths_log()
    assert got == orc.cached_paths_log()
    assert len(got) > 0


@pytest.mark.parametrize("name", ["complete30_ms", "complete25_dir", "sparse300_ms", "sparse5000_hbm", "dense4400_hbm"])
def test_minplus_latencies_equal_table(name):
    """shd_topology_latency_table_fw (blocked min-plus Floyd-Warshall, 64 x 64
    LDS tiles): the latency half of the table, bit for bit, self paths and
    directed graphs included; no lookup side effects."""
    import torch
    gml, H = GRAPHS[name]
    top, orc, _, _ = make_pair(gml, H)
    lat, rel, sv = top.table()
    A = len(sv)
    d = torch.empty(A * A, dtype=torch.float64, device="cuda")
    top.latency_table_fw(d.data_ptr())
    fw = d.cpu().numpy().reshape(A, A)
    assert np.array_equal(bits(fw), bits(lat)), name


@pytest.mark.parametrize("name", ["complete30_ms", "complete25_dir", "sparse300_ms", "sparse5000_hbm", "dense4400_hbm"])
def test_frontier_latencies_equal_table(name):
    """shd_topology_latency_rows_frontier (bucketed frontier SSSP, one wave per
    source): the latency half of the table, bit for bit, self paths and
    directed graphs included -- all rows, and a sub-range written from its
    first row."""
    import torch
    gml, H = GRAPHS[name]
    top, orc, _, _ = make_pair(gml, H)
    lat, rel, sv = top.table()
    A = len(sv)
    d = torch.full((A * A,), 7.0, dtype=torch.float64, device="cuda")
    top.latency_rows_frontier(0, A, d.data_ptr())
    assert np.array_equal(bits(d.cpu().numpy().reshape(A, A)), bits(lat)), name
    lo, hi = A // 3, A // 3 + max(1, A // 4)
    d2 = torch.full(((hi - lo) * A,), 7.0, dtype=torch.float64, device="cuda")
    top.latency_rows_frontier(lo, hi, d2.data_ptr())
    assert np.array_equal(bits(d2.cpu().numpy().reshape(hi - lo, A)), bits(lat[lo:hi])), name


@pytest.mark.parametrize("wmax", [3348, 3349])
def test_frontier_largest_edge_latency(wmax):
    """The frontier kernel's bucket ring lives in LDS: edge latencies up to
    3,348 ms (every row equal to the table's latencies), one more declines
    with -ENOTSUP (shdnet.h)."""
    import torch
    gml = synth.sparse_graph_gml(300, 0x5EED0F01, max_ms=wmax - 1)
    gml = gml.replace('latency "1 ms"', f'latency "{wmax} ms"', 1)
    assert f'"{wmax} ms"' in gml
    top, orc, _, _ = make_pair(gml, 400)
    lat, rel, sv = top.table()
    A = len(sv)
    d = torch.full((A * A,), 7.0, dtype=torch.float64, device="cuda")
    if wmax <= 3348:
        top.latency_rows_frontier(0, A, d.data_ptr())
        assert np.array_equal(bits(d.cpu().numpy().reshape(A, A)), bits(lat))
    else:
        from shadow_amd._lib import ShdError
        with pytest.raises(ShdError) as ei:
            top.latency_rows_frontier(0, A, d.data_ptr())
        assert ei.value.code == -95  # ENOTSUP


def test_frontier_needs_whole_ms():
    """Fractional-ms latencies: the frontier entry declines (-ENOTSUP)."""
    import torch
    gml, H = GRAPHS["sparse300_ns"]
    top, _, _, _ = make_pair(gml, H)
    A = top.slot_count()
    d = torch.empty(A * A, dtype=torch.float64, device="cuda")
    from shadow_amd._lib import ShdError
    with pytest.raises(ShdError) as ei:
        top.latency_rows_frontier(0, A, d.data_ptr())
    assert ei.value.code == -95  # ENOTSUP


def test_minplus_needs_whole_ms():
    """Fractional-ms latencies: the min-plus entry declines (-ENOTSUP)."""
    import torch
    gml, H = GRAPHS["complete40_ns"]
    top, _, _, _ = make_pair(gml, H)
    A = top.slot_count()
    d = torch.empty(A * A, dtype=torch.float64, device="cuda")
    from shadow_amd._lib import ShdError
    with pytest.raises(ShdError) as ei:
        top.latency_table_fw(d.data_ptr())
    assert ei.value.code == -95  # ENOTSUP


@pytest.mark.timeout(60)
def test_large_complete_graph_list_handles():
    """A complete graph with more than 2^23 incidence entries (V = 3,000: 9M):
    list starts above 2^23 in the 24-bit handles (read unsigned); sampled
    rows against the oracle, the min-plus latencies against the table."""
    import torch
    gml = synth.complete_graph_gml(3000, 0x5EED0081)
    top, orc, _, _ = make_pair(gml, 6000)
    lat, rel, sv = top.table()
    for i in list(range(0, len(sv), 97)) + [len(sv) - 1]:
        ol, orl = orc.row(int(sv[i]), sv)
        assert np.array_equal(bits(lat[i]), bits(ol)), i
        assert np.array_equal(bits(rel[i]), bits(orl)), i
    A = len(sv)
    d = torch.empty(A * A, dtype=torch.float64, device="cuda")
    top.latency_table_fw(d.data_ptr())
    assert np.array_equal(bits(d.cpu().numpy().reshape(A, A)), bits(lat))

