"""CPU-only checks of the product library: it loads, exports every symbol
include/shdnet.h declares, and its host-side logic (GML load, validation,
attachment) agrees with the oracle.  No GPU compute is called here."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import oracle_ctypes as O
from shadow_amd import ShdError, Topology, _lib, scenario, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    text = open(os.path.join(ROOT, "include", "shdnet.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(shd_\w+)\s*\(", text, re.M)))


def test_library_exports_every_header_symbol():
    lib = _lib.lib()
    syms = header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), s
    # every exported prototype in _lib matches a header declaration
    assert set(_lib.PROTOS) == set(syms)


def test_no_oracle_in_product():
    """The product never imports, links or calls the oracle."""
    for dp, _, fs in os.walk(os.path.join(ROOT, "shadow_amd")):
        for f in fs:
            if f.endswith((".py", ".c", ".h", ".hip", "Makefile")):
                txt = open(os.path.join(dp, f), errors="ignore").read()
                assert not re.search(r"oracle_ctypes|liboracle|oracle/|import oracle|orc_\w+\(", txt), f


@pytest.mark.parametrize("gml", [synth.ONE_GBIT_SWITCH_GML, synth.complete_graph_gml(12, 5),
                                 synth.sparse_graph_gml(300, 9, directed=True)])
def test_topology_load_and_info(gml):
    t = Topology(gml)
    o = O.OracleTopology(gml)
    info = t.info()
    assert info["vertices"] == o.V
    assert info["directed"] == o.directed
    assert info["complete"] == o.complete


INVALID = [
    synth.complete_graph_gml(4, 7).replace('latency "', 'latency "-', 1),
    synth.complete_graph_gml(4, 7).replace("packet_loss 0", "packet_loss 2", 1),
    synth.complete_graph_gml(4, 7).replace("bandwidth_up", "weight", 1),
    synth.complete_graph_gml(4, 7).replace('"1 Gbit"', '"1 Kbit"', 1),   # 1000 bit/s -> 0 KiB/s
    synth.complete_graph_gml(4, 7).replace('latency "', 'latency "1.5', 1),
    "graph [\n  node [\n    id 0\n  ]\n]",
    "graph [ node [ id 0 bandwidth_up \"1 Gbit\" bandwidth_down \"1 Gbit\" ] node [ id 0 bandwidth_up "
    "\"1 Gbit\" bandwidth_down \"1 Gbit\" ] edge [ source 0 target 0 latency \"1 ms\" packet_loss 0 ] ]",
    synth.sparse_graph_gml(10, 3).split("  edge [")[0] + "]\n",
    "not a graph",
]


@pytest.mark.parametrize("i", range(len(INVALID)))
def test_invalid_graphs_rejected_like_oracle(i):
    with pytest.raises(ValueError):
        O.OracleTopology(INVALID[i])
    with pytest.raises(ShdError):
        Topology(INVALID[i])


def test_incomplete_graph_needs_shortest_path():
    g = synth.sparse_graph_gml(30, 3)
    Topology(g, use_shortest_path=True)
    with pytest.raises(ShdError):
        Topology(g, use_shortest_path=False)


def test_attach_matches_oracle_with_hints():
    """Hints, city/country filters, exact IP match and longest-prefix match
    (topology.c:2024-2216) on a graph with vertex IPs and codes."""
    V = 40
    nodes = []
    for v in range(V):
        ip = f"10.{v % 4}.{v}.1" if v % 3 else ""
        nodes.append(f"  node [\n    id {v}\n" + (f"    ip_address \"{ip}\"\n" if ip else "")
                     + f"    city_code \"c{v % 5}\"\n    country_code \"K{v % 2}\"\n"
                     + "    bandwidth_up \"1 Gbit\"\n    bandwidth_down \"1 Gbit\"\n  ]\n")
    edges = "".join(f"  edge [\n    source {v}\n    target {(v + 1) % V}\n    latency \"{v + 1} ms\"\n"
                    f"    packet_loss 0.0\n  ]\n" for v in range(V))
    gml = "graph [\n  directed 0\n" + "".join(nodes) + edges + "]\n"
    t = Topology(gml)
    o = O.OracleTopology(gml)
    ips = synth.host_ips(64)
    hints = [(None, None, None), ("10.1.5.1", None, None), ("10.2.77.9", None, None), (None, "c3", None),
             (None, "zz", "K1"), ("10.0.3.1", "c3", None), ("0.0.0.0", None, None), (None, "C2", "k0"),
             ("127.0.0.1", None, None), ("10.3.200.1", None, "K0")]
    for h in range(64):
        ip_hint, city, country = hints[h % len(hints)]
        a = t.attach(h, int(ips[h]), 1000 + h, ip_hint, city, country)
        b = o.attach(h, int(ips[h]), 1000 + h, ip_hint, city, country)
        assert a == b, (h, ip_hint, city, country)


def test_product_unit_parser_matches_reference_tests():
    """csrc/units.c (the parser the GML loader uses) against the cases and
    values the reference's own Rust tests state (units.rs:579-775), the same
    fixture the oracle is pinned by."""
    import json
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "units_cases.json")))
    lib = _lib.lib()
    out = C.c_uint64()
    for fn, key in ((lib.shd_parse_time_ns, "time_ns"), (lib.shd_parse_bandwidth_bits, "bandwidth_bits")):
        for s, want in g[key]:
            rc = fn(s.encode(), C.byref(out))
            if want < 0:
                assert rc != 0, s
            else:
                assert rc == 0 and out.value == want, (s, want, out.value)
    assert len(g["time_ns"]) >= 10 and any(w < 0 for _, w in g["time_ns"])


def test_seed_chain_matches_reference_fixture():
    import json
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "ref_random_pq.json")))
    for c in g["chains"]:
        assert list(scenario.host_seeds(c["seed"], len(c["hosts"]))) == c["hosts"]


def test_packet_batch_prestates():
    """rng pre-states advance one rand_r per earlier send of the same host."""
    seeds = np.array([1, 2, 3, 4], dtype=np.uint32)
    pk = synth.packet_batch(200, 4, 5, 0, 1000, seeds)
    cur = {h: int(seeds[h]) for h in range(4)}
    for p in pk:
        h = int(p["src_host"])
        assert int(p["rng_state"]) == cur[h]
        _, cur[h] = scenario._rand_r(cur[h])
