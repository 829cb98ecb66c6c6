#!/usr/bin/env python3
"""Generates the committed golden fixtures under tests/golden/ (TEST INFRASTRUCTURE).

Run in the build container (needs /root/reference and networkx):
    make -C oracle ref && python oracle/gen_golden.py

Fixtures produced (all data, no reference source text):
  ref_random_pq.json  outputs of the REFERENCE's own utility/random.c and
                      utility/priority_queue.c (compiled from /root/reference
                      by oracle/Makefile into oracle/_ref/ref_driver).
  units_cases.json    unit-string cases and expected values stated by the
                      reference's Rust tests (core/support/units.rs:579-775)
                      plus the graph strings used by the reference test configs.
  selfloop_cases.json the single-vertex graphs every reference test uses
                      (1_gbit_switch configuration.rs:728-742; tcp/*-lossy.yaml)
                      with the values the reference code fixes for them.
  nx_tables.json      fp64 path latencies (and reliabilities where the shortest
                      path is unique) from networkx 3.4.2 Dijkstra on small
                      synthetic graphs: an independent, tie-free check of the
                      oracle's igraph restatement.
"""
import json
import os
import subprocess
import sys

import networkx as nx

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
from shadow_amd import synth  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")


def ref_random_pq():
    exe = os.path.join(HERE, "_ref", "ref_driver")
    out = subprocess.check_output([exe], text=True)
    data = json.loads(out)
    data["_source"] = "oracle/_ref/ref_driver (reference src/main/utility/random.c + priority_queue.c)"
    with open(os.path.join(GOLD, "ref_random_pq.json"), "w") as f:
        json.dump(data, f)


def units_cases():
    S = 1_000_000_000
    time_cases = [
        # units.rs:579-628 (test_parse_string) -> converted to ns (parse_time_nanosec)
        ["10", 10 * S], ["10 s", 10 * S], ["10s", 10 * S], ["10   s", 10 * S], ["10sec", 10 * S],
        ["10  m", 600 * S], ["10  min", 600 * S], ["10 ms", 10_000_000], ["10 μs", 10_000],
        ["10 millisecond", 10_000_000], ["10 milliseconds", 10_000_000],
        ["-10 ms", -1], ["abc 10 ms", -1], ["10.5 ms", -1], ["10 abc", -1],
        # units.rs:760-766 conversions
        ["70 min", 4200 * S], ["1 hour", 3600 * S],
        # strings used by the reference graphs / docs
        ["1 ms", 1_000_000], ["50 ms", 50_000_000], ["123 ns", 123], ["5 us", 5000],
        ["0 ms", 0], ["+7 ms", 7_000_000], ["", -1], [" 10 ms ", -1], ["10 ms ", 10_000_000],
        ["18446744073709551615 ns", -1], ["9223372036854775807 ns", 9223372036854775807],
        ["3000000 h", -1], ["2 hrs", 7200 * S], ["10 nanoseconds", 10],
    ]
    bw_cases = [
        # units.rs:680-708 (BitsPerSec) -> bits/s (parse_bandwidth)
        ["10", 10], ["10 bit", 10], ["10bit", 10], ["10   bit", 10], ["10  Kbit", 10_000],
        ["10 Kibit", 10_240], ["10 Mbit", 10_000_000], ["10 megabit", 10_000_000],
        ["10 megabits", 10_000_000], ["-10 Kbit", -1], ["abc 10 Kbit", -1], ["10.5 Kbit", -1],
        ["10 abc", -1], ["10 mbit", -1],
        # units.rs:748-752 conversion, graph strings
        ["1024 Kbit", 1_024_000], ["1 Gbit", 1_000_000_000], ["81920 Kibit", 83_886_080],
    ]
    with open(os.path.join(GOLD, "units_cases.json"), "w") as f:
        json.dump({"time_ns": time_cases, "bandwidth_bits": bw_cases,
                   "_source": "core/support/units.rs:579-775 (expected values as the Rust tests state them)"},
                  f, ensure_ascii=False, indent=0)


def selfloop_cases():
    lossy = """graph [
  directed 0
  node [
    id 0
    country_code "US"
    bandwidth_down "81920 Kibit"
    bandwidth_up "81920 Kibit"
  ]
  edge [
    source 0
    target 0
    latency "50 ms"
    packet_loss 0.25
  ]
]"""
    lossless = lossy.replace("packet_loss 0.25", "packet_loss 0.0")
    cases = [
        {"name": "1_gbit_switch", "gml": synth.ONE_GBIT_SWITCH_GML, "latency_ms": 1.0, "reliability": 1.0,
         "delay_ns": 1_000_000, "bw_kibps": 122070,
         "_source": "configuration.rs:728-742; getting_started_basic.md"},
        {"name": "tcp-lossy", "gml": lossy, "latency_ms": 50.0, "reliability": 0.75, "delay_ns": 50_000_000,
         "bw_kibps": 10240, "_source": "test/tcp/tcp-blocking-lossy.yaml:1-21"},
        {"name": "tcp-lossless", "gml": lossless, "latency_ms": 50.0, "reliability": 1.0,
         "delay_ns": 50_000_000, "bw_kibps": 10240, "_source": "test/tcp/tcp-blocking-lossless.yaml"},
    ]
    with open(os.path.join(GOLD, "selfloop_cases.json"), "w") as f:
        json.dump(cases, f, indent=1)


def gml_to_nx(text):
    """Tiny reader for the synthetic GML dialect (generated here, known shape)."""
    directed = "directed 1" in text.split("node", 1)[0]
    G = nx.DiGraph() if directed else nx.Graph()
    for blk in text.split("node [")[1:]:
        vid = int(blk.split("id", 1)[1].split()[0])
        G.add_node(vid)
    for blk in text.split("edge [")[1:]:
        f = blk.split()
        s = int(f[f.index("source") + 1])
        t = int(f[f.index("target") + 1])
        lat = blk.split("latency \"", 1)[1].split("\"", 1)[0]
        val, unit = lat.split()
        ns = int(val) * {"ms": 1_000_000, "ns": 1}[unit]
        loss = float(f[f.index("packet_loss") + 1])
        if s == t:
            continue
        G.add_edge(s, t, weight=ns / 1000000.0, rel=1.0 - loss)
    return G


def nx_tables():
    graphs = [
        ("complete30_ms", synth.complete_graph_gml(30, 0x5EED0001)),
        ("complete30_ns", synth.complete_graph_gml(30, 0x5EED0011, ns_variant=True)),
        ("sparse200_ns", synth.sparse_graph_gml(200, 0x5EED0002, ns_variant=True)),
        ("sparse200_ms", synth.sparse_graph_gml(200, 0x5EED0012)),
        ("sparse150_dir_ns", synth.sparse_graph_gml(150, 0x5EED0022, ns_variant=True, directed=True)),
    ]
    out = []
    for name, gml in graphs:
        G = gml_to_nx(gml)
        V = G.number_of_nodes()
        lat = [[None] * V for _ in range(V)]
        rel = [[None] * V for _ in range(V)]
        for s in range(V):
            pred, dist = nx.dijkstra_predecessor_and_distance(G, s)
            for t in range(V):
                if t == s:
                    continue
                lat[s][t] = dist[t]
                # reliability only where the fp64 shortest path is unique
                path, v, unique = [t], t, True
                while v != s:
                    if len(pred[v]) != 1:
                        unique = False
                        break
                    v = pred[v][0]
                    path.append(v)
                if unique:
                    path.reverse()
                    r = 1.0
                    for a, b in zip(path, path[1:]):
                        r *= G[a][b]["rel"]
                    rel[s][t] = r
        out.append({"name": name, "gml": gml, "V": V, "lat": lat, "rel": rel})
    with open(os.path.join(GOLD, "nx_tables.json"), "w") as f:
        json.dump({"_source": "networkx %s dijkstra_predecessor_and_distance" % nx.__version__,
                   "graphs": out}, f)


if __name__ == "__main__":
    os.makedirs(GOLD, exist_ok=True)
    ref_random_pq()
    units_cases()
    selfloop_cases()
    nx_tables()
    print("golden fixtures written to", GOLD)
