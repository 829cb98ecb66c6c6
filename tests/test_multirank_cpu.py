"""N>1 path on CPU: world_size-2 (and 3) gloo runs of the destination-owner
exchange.  Each rank decides its own senders' packets (the oracle stands in
for the GPU packet-scatter output here: same CSR-grouped events), exchanges by
destination owner, regroups; the union over ranks must equal a single-rank
round over all packets, per destination, in event_compare order."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_ctypes as O
from shadow_amd import exchange, scenario, synth

H = 48
GML = synth.complete_graph_gml(16, 0x5EED0061, ns_variant=True)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_with_rows():
    orc = O.OracleTopology(GML)
    ips, st, verts = scenario.register_hosts(orc, H, 1)
    sv = np.unique(verts).astype(np.int32)
    lat = np.empty((len(sv), len(sv)))
    rel = np.empty((len(sv), len(sv)))
    for i, s in enumerate(sv):
        lat[i], rel[i] = orc.row(int(s), sv)
    orc.preload(sv, lat, rel)  # rows released in slot order (touch_all)
    return orc, ips, st


def _rank_packets(rank, world, st):
    lo, hi = rank * H // world, (rank + 1) * H // world
    return synth.packet_batch(3000, H, 0x5EED0400 + rank, 100_000_000, 10_000_000, st, hosts_lo=lo, hosts_hi=hi)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    orc, ips, st = _oracle_with_rows()
    pk = _rank_packets(rank, world, st)
    out, status, mt = orc.round(ips, pk, 110_000_000, 10**15)
    offs = np.zeros(H + 1, dtype=np.int64)
    offs[1:] = np.cumsum(np.bincount(out["dst_host"], minlength=H))
    ev = torch.from_numpy(out.view(np.uint8).copy())
    bounds = exchange.owner_bounds(H, world)
    recv, n, counts = exchange.exchange_events(ev, torch.from_numpy(offs), bounds)
    got = recv[:n * 32].numpy().view(synth.DELIV_DTYPE)
    lo, hi = bounds[rank], bounds[rank + 1]
    assert ((got["dst_host"] >= lo) & (got["dst_host"] < hi)).all()
    # regroup (the GPU does this with shd_deliv_sort_device)
    got = got[np.lexsort((got["seq"], got["src_host"], got["time"], got["dst_host"]))]
    mts = torch.tensor([mt], dtype=torch.float64)
    dist.all_reduce(mts, op=dist.ReduceOp.MIN)
    q.put((rank, got.tobytes(), float(mts.item())))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_gloo_matches_single_rank(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    merged = np.concatenate([np.frombuffer(b, dtype=synth.DELIV_DTYPE) for _, b, _ in res])
    # single rank: all packets of every rank, one round
    orc, ips, st = _oracle_with_rows()
    allpk = np.concatenate([_rank_packets(r, world, st) for r in range(world)])
    ref, _, mt = orc.round(ips, allpk, 110_000_000, 10**15)
    for k in ("dst_host", "time", "src_host", "seq"):
        assert np.array_equal(merged[k], ref[k]), k
    assert all(m == mt for _, _, m in res)
