#!/usr/bin/env python3
"""How many routing-table entries are decided by igraph's heap order?

For each source s and target d != s, counts the predecessors u of d with
dist(s,u) + w(u,d) == dist(s,d) (exact: the synthetic latencies are integer
ms, so fp64 sums are exact).  With more than one, the path -- and therefore
the reliability product -- is chosen by the pop order of igraph's binary
heap, which a distance-only algorithm (blocked min-plus
Floyd-Warshall, frontier/delta-stepping SSSP) does not reproduce.
Usage: scripts/tie_stats.py [c1|c2] [nsources]"""
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from shadow_amd import synth  # noqa: E402
from scipy.sparse import csr_matrix  # noqa: E402
from scipy.sparse.csgraph import dijkstra  # noqa: E402


def parse(gml):
    src, dst, w = [], [], []
    V = gml.count("node [")
    for blk in gml.split("edge [")[1:]:
        f = {}
        for line in blk.splitlines():
            p = line.strip().split(None, 1)
            if len(p) == 2:
                f[p[0]] = p[1].strip('"')
        lat = f["latency"].split()
        ms = float(lat[0]) / (1e6 if lat[1] == "ns" else 1.0)
        a, b = int(f["source"]), int(f["target"])
        if a != b:
            src += [a, b]; dst += [b, a]; w += [ms, ms]
    return V, np.array(src), np.array(dst), np.array(w)


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c1"
    ns = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    gml = (synth.complete_graph_gml(1000, 0x5EED0001) if cfg == "c1" else
           synth.sparse_graph_gml(20000, 0x5EED0002) if cfg == "c2" else synth.sparse_graph_gml(100000, 0x5EED0004))
    V, s, d, w = parse(gml)
    M = csr_matrix((w, (s, d)), shape=(V, V))
    srcs = np.arange(0, V, max(1, V // ns))[:ns]
    D = dijkstra(M, directed=True, indices=srcs)
    tied_pairs = pairs = tied_rows = amb_pairs = amb_rows = 0
    for i, so in enumerate(srcs):
        dist = D[i]
        tight = np.isclose(dist[s] + w, dist[d], rtol=0, atol=1e-9)  # exact for integer ms
        npred = np.bincount(d[tight], minlength=V)
        npred[so] = 0
        t = int((npred > 1).sum())
        tied_pairs += t
        pairs += V - 1
        tied_rows += t > 0
        # igraph's parent = the FIRST POPPED tight predecessor; pop order is by
        # distance, so only tight predecessors of equal (minimal) distance are
        # decided by the heap: count those vertices
        ts, td = s[tight], d[tight]
        du = dist[ts]
        mind = np.full(V, np.inf)
        np.minimum.at(mind, td, du)
        nmin = np.bincount(td[du == mind[td]], minlength=V)
        nmin[so] = 0
        a = int((nmin > 1).sum())
        amb_pairs += a
        amb_rows += a > 0
    print(f"{cfg}: V={V}, {len(srcs)} sources: {tied_pairs}/{pairs} = {tied_pairs / pairs:.1%} of (s,d) pairs "
          f"have >1 shortest-path predecessor; {tied_rows}/{len(srcs)} rows contain at least one")
    print(f"{cfg}: {amb_pairs}/{pairs} = {amb_pairs / pairs:.2%} of vertices have >1 shortest-path predecessor of "
          f"EQUAL (minimal) distance -- the only ones whose parent needs the heap's pop order; "
          f"{amb_rows}/{len(srcs)} rows contain at least one")


if __name__ == "__main__":
    main()
