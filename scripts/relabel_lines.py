#!/usr/bin/env python3
"""Routing C4 (V=100k): distinct 128-B lines (8 16-B records) among each
vertex's neighbours -- the record gathers of one pop -- under the product's
labelling and under RCM / BFS-from-the-hub / degree-descending relabellings.
CPU only.  Usage: relabel_lines.py [seed]"""
import sys, numpy as np, re
sys.path.insert(0,'/root/repo')
from shadow_amd import synth
from scipy.sparse import csr_matrix
from scipy.sparse.csgraph import reverse_cuthill_mckee, breadth_first_order
V=100_000
gml=synth.sparse_graph_gml(V, int(sys.argv[1],0) if len(sys.argv)>1 else 0x5EED0004)
src=np.array([int(x) for x in re.findall(r'source (\d+)', gml)]); dst=np.array([int(x) for x in re.findall(r'target (\d+)', gml)])
m=src!=dst; src,dst=src[m],dst[m]
A=csr_matrix((np.ones(2*len(src)),(np.r_[src,dst],np.r_[dst,src])),shape=(V,V))
deg=np.diff(A.indptr)
print('edges',len(src),'avg deg',deg.mean(),'max',deg.max())
def lines(perm):  # perm[v] = new id
    tot=0
    for u in range(V):
        nb=A.indices[A.indptr[u]:A.indptr[u+1]]
        tot+=len(np.unique(perm[nb]//8))
    return tot/V
ident=np.arange(V)
print('identity lines/pop', lines(ident))
rcm=reverse_cuthill_mckee(A,symmetric_mode=True); p=np.empty(V,int); p[rcm]=np.arange(V); print('rcm', lines(p))
order=breadth_first_order(A, int(np.argmax(deg)), directed=False, return_predecessors=False); p=np.empty(V,int); p[order]=np.arange(V); print('bfs(hub)', lines(p))
od=np.argsort(-deg,kind='stable'); p=np.empty(V,int); p[od]=np.arange(V); print('degree desc', lines(p))
