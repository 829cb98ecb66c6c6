"""Multi-GPU rounds through the C entry points, rehearsed with
world sizes 2 and 3 on one GPU (every rank on cuda:0, the gloo-backed
TorchTransport; the 8-GPU node runs the same code over RCCL).

replicated: rank r builds rows [row_bounds[r], row_bounds[r+1]) of the
  table and shd_topology_allgather_rows completes it on every rank (the
  full-matrix all-gather of §8e, through the transport's allgatherv); every
  rank then decides its own senders' packets (shd_round_process_device), and
  shd_round_exchange sends each event to its destination's owner rank, which
  regroups it with shd_deliv_sort_device.  The gathered table is checked
  bitwise against the oracle's rows.
fused: the same table, then shd_round_process_exchange: decide, group by
  destination without sorting, ship 24-B wire records, merge at the owner.
sharded: rank r builds and holds only rows [row_bounds[r], row_bounds[r+1])
  (shd_topology_adopt_table_shard_device_resident); shd_round_route_records
  first moves every record to the rank holding the row that answers it,
  which decides it; then the same exchange.
Either way the union over ranks must equal the oracle's single round over
all ranks' packets: the same events, per destination in event_compare order,
and the same min delivered time.
"""
import numpy as np
import pytest

from rank_procs import run_ranks

pytestmark = pytest.mark.gpu

H = 300
BARRIER, END = 110_000_000, 10**15


def _gml():
    from shadow_amd import synth
    return synth.sparse_graph_gml(250, 0x5EED0801, ns_variant=True)


def _packets(rank, world, st):
    from shadow_amd import synth
    lo, hi = rank * H // world, (rank + 1) * H // world
    return synth.packet_batch(4000, H, 0x5EED0810 + rank, 100_000_000, 10_000_000, st, hosts_lo=lo, hosts_hi=hi)


def _worker(rank, world, mode):
    import torch
    import torch.distributed as dist

    from shadow_amd import Topology, scenario, synth
    from shadow_amd.transport import TorchTransport
    torch.cuda.set_device(0)
    top = Topology(_gml())
    ips, st, verts = scenario.register_hosts(top, H, seed=1)
    A = top.slot_count()
    row_bounds = [r * A // world for r in range(world + 1)]
    host_bounds = [r * H // world for r in range(world + 1)]
    pk = _packets(rank, world, st)
    xp = TorchTransport(device=torch.device("cuda", 0))
    table = b""
    if mode in ("replicated", "fused"):
        lo, hi = row_bounds[rank], row_bounds[rank + 1]
        tab = torch.zeros(A * A * 2, dtype=torch.float64, device="cuda")
        if hi > lo:
            top.build_rows_device(lo, hi, tab.data_ptr())
        torch.cuda.synchronize()
        xp.register(tab)
        top.allgather_rows(xp, tab.data_ptr(), row_bounds)
        table = tab.cpu().numpy().tobytes()
        top.adopt_table_device(tab.data_ptr())
        top.touch_all()
        recs = torch.from_numpy(pk.view(np.uint8)).cuda()
        n = len(pk)
    else:
        lo, hi = row_bounds[rank], row_bounds[rank + 1]
        shard = torch.empty(max(hi - lo, 1) * A * 2, dtype=torch.float64, device="cuda")
        if hi > lo:
            top.build_rows_device(lo, hi, shard.data_ptr() - lo * A * 16)
        torch.cuda.synchronize()
        mn = torch.tensor([top.shard_min_latency(shard.data_ptr(), lo, hi)], dtype=torch.float64)
        mn[mn < 0] = float("inf")
        dist.all_reduce(mn, op=dist.ReduceOp.MIN)
        top.adopt_table_shard_device_resident(shard.data_ptr(), lo, hi, float(mn.item()))
        src = torch.from_numpy(pk.view(np.uint8)).cuda()
        scratch = torch.empty_like(src)
        cap = 4000 * world
        recs = torch.empty(cap * 32, dtype=torch.uint8, device="cuda")
        xp.register(scratch, recs)
        n = top.route_records(xp, src.data_ptr(), len(pk), row_bounds, scratch.data_ptr(), recs.data_ptr(), cap)
    if mode == "fused":  # decide + group + exchange + merge in one call (24-B wire records)
        cap = 4000 * world
        d_send = torch.empty(max(n, 1) * 24, dtype=torch.uint8, device="cuda")
        d_wrecv = torch.empty(cap * 24, dtype=torch.uint8, device="cuda")
        d_final = torch.empty(cap * 32, dtype=torch.uint8, device="cuda")
        d_status = torch.empty(max(n, 1), dtype=torch.uint8, device="cuda")
        d_cnt = torch.empty(2, dtype=torch.int64, device="cuda")
        mine = host_bounds[rank + 1] - host_bounds[rank]
        d_final_off = torch.empty(mine + 1, dtype=torch.int32, device="cuda")
        xp.register(d_send, d_wrecv)
        nrecv = top.process_exchange(xp, recs.data_ptr(), n, BARRIER, END, 0, host_bounds, d_send.data_ptr(),
                                     d_status.data_ptr(), d_cnt.data_ptr(), d_wrecv.data_ptr(), cap,
                                     d_final.data_ptr(), d_final_off.data_ptr())
        status = d_status.cpu().numpy()[:n]
        got = d_final.cpu().numpy().view(synth.DELIV_DTYPE)[:nrecv].copy()
        offs = d_final_off.cpu().numpy()
        assert offs[-1] == nrecv
        assert np.array_equal(np.diff(offs), np.bincount(got["dst_host"] - host_bounds[rank], minlength=mine))
        mt = torch.tensor([int(d_cnt.cpu().numpy().view(np.uint64)[1])], dtype=torch.float64)
        dist.all_reduce(mt, op=dist.ReduceOp.MIN)
        return rank, got.tobytes(), float(mt.item()), int((status == 1).sum()), table
    cap = max(n, 1) * world
    d_out = torch.empty(max(n, 1) * 32, dtype=torch.uint8, device="cuda")
    d_off = torch.empty(H + 1, dtype=torch.int32, device="cuda")
    d_status = torch.empty(max(n, 1), dtype=torch.uint8, device="cuda")
    d_cnt = torch.empty(2, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    top.process_device(recs.data_ptr(), n, BARRIER, END, 0, d_out.data_ptr(), d_off.data_ptr(),
                       d_status.data_ptr(), d_cnt.data_ptr(), 0)
    torch.cuda.synchronize()
    status = d_status.cpu().numpy()[:n]
    assert (status != 0xFF).all(), "a record reached a rank without its answering row"
    d_recv = torch.empty(4000 * world * 32, dtype=torch.uint8, device="cuda")
    d_final = torch.empty_like(d_recv)
    mine = host_bounds[rank + 1] - host_bounds[rank]
    d_final_off = torch.empty(mine + 1, dtype=torch.int32, device="cuda")
    xp.register(d_out, d_recv)
    nrecv = top.exchange(xp, d_out.data_ptr(), d_off.data_ptr(), host_bounds, d_recv.data_ptr(), 4000 * world,
                         d_final.data_ptr(), d_final_off.data_ptr())
    got = d_final.cpu().numpy().view(synth.DELIV_DTYPE)[:nrecv].copy()
    offs = d_final_off.cpu().numpy()
    assert offs[-1] == nrecv
    assert np.array_equal(np.diff(offs), np.bincount(got["dst_host"] - host_bounds[rank], minlength=mine))
    mt = torch.tensor([int(d_cnt.cpu().numpy().view(np.uint64)[1])], dtype=torch.float64)
    dist.all_reduce(mt, op=dist.ReduceOp.MIN)
    return rank, got.tobytes(), float(mt.item()), int((status == 1).sum()), table


@pytest.mark.timeout(60)
@pytest.mark.parametrize("mode,world,runs", [("replicated", 2, "1"), ("replicated", 3, "1"), ("sharded", 2, "1"),
                                             ("sharded", 3, "1"), ("replicated", 3, "0"), ("sharded", 2, "0"),
                                             ("fused", 2, "1"), ("fused", 3, "1")])
def test_multirank_round_through_c_abi(world, mode, runs, tmp_path):
    """runs "1": the owner merges the W received destination-sorted runs in
    place (default); "0": it re-scatters them into destination slabs (the
    round-2 regroup, SHD_XCHG_RUNS=0)."""
    import oracle_ctypes as O
    from shadow_amd import scenario, synth
    res = run_ranks(_worker, world, tmp_path, args=(mode,), env={"SHD_XCHG_RUNS": runs}, deadline=45)
    merged = np.concatenate([np.frombuffer(b, dtype=synth.DELIV_DTYPE) for _, b, *_ in res])
    orc = O.OracleTopology(_gml())
    ips, st, verts = scenario.register_hosts(orc, H, 1)
    sv = np.unique(verts).astype(np.int32)
    lat, rel = orc.rows_parallel(sv, sv, 8)
    if mode in ("replicated", "fused"):  # every rank's all-gathered table == the oracle's rows
        want = np.stack([lat, rel], axis=-1).tobytes()
        assert all(r[4] == want for r in res)
    orc.preload(sv, lat, rel)  # every row released in slot order, as touch_all / the shard adoption
    allpk = np.concatenate([_packets(r, world, st) for r in range(world)])
    ref, status, mt = orc.round(ips, allpk, BARRIER, END)
    assert len(merged) == len(ref) == sum(r[3] for r in res)
    for k in ("dst_host", "time", "src_host", "seq"):
        assert np.array_equal(merged[k], ref[k]), k
    assert all(r[2] == float(mt) for r in res)
