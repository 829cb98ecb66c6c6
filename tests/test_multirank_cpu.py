"""The N>1 transport on CPU: world_size-2 and 3 gloo runs of the
TorchTransport collectives exactly as libshdnet calls them (through the
ShdTransport function pointers): the count all-to-all and the contiguous
per-peer block all-to-all(v) that shd_round_exchange / _route_records issue,
and the in-place all-gather(v) of shd_topology_allgather_rows (equal blocks:
one all_gather; unequal or empty blocks: one broadcast per rank).
The GPU side (kernels, regroup, row routing) runs in test_multirank_gpu.py."""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _blocks(rank, world):
    """Rank's send blocks: to peer r, (rank + 1) * (r + 2) records of 32 bytes."""
    rng = np.random.default_rng(100 + rank)
    sizes = [(rank + 1) * (r + 2) for r in range(world)]
    data = rng.integers(0, 256, sum(sizes) * 32, dtype=np.uint8)
    return sizes, data


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from shadow_amd.transport import TorchTransport
    dist.init_process_group("gloo", rank=rank, world_size=world)
    xp = TorchTransport(device=torch.device("cpu"))
    st = xp.struct
    assert st.rank == rank and st.world == world
    sizes, data = _blocks(rank, world)
    send = (C.c_uint64 * world)(*sizes)
    recv = (C.c_uint64 * world)()
    assert st.alltoall_u64(None, send, recv) == 0, xp.error
    rsizes = list(recv)
    src = torch.from_numpy(data.copy())
    dst = torch.zeros(sum(rsizes) * 32 + 64, dtype=torch.uint8)
    xp.register(src, dst)
    sb = (C.c_uint64 * world)(*[x * 32 for x in sizes])
    rb = (C.c_uint64 * world)(*[x * 32 for x in rsizes])
    assert st.alltoallv(None, src.data_ptr(), sb, dst.data_ptr(), rb, None) == 0, xp.error
    # allgatherv in place: rank r owns rows [bounds[r], bounds[r+1]) of a
    # table of 48-byte rows; two layouts (equal, ragged with an empty block)
    gathered = []
    for bounds in (_row_bounds(world, equal=True), _row_bounds(world, equal=False)):
        tab = torch.zeros(bounds[-1] * 48, dtype=torch.uint8)
        tab[bounds[rank] * 48:bounds[rank + 1] * 48] = torch.from_numpy(_rows(rank, bounds))
        xp.register(tab)
        offs = (C.c_uint64 * (world + 1))(*[b * 48 for b in bounds])
        assert st.allgatherv(None, tab.data_ptr(), offs, None) == 0, xp.error
        gathered.append(tab.numpy().tobytes())
    q.put((rank, rsizes, dst[:sum(rsizes) * 32].numpy().tobytes(), gathered))
    dist.destroy_process_group()


def _row_bounds(world, equal):
    if equal:
        return [5 * r for r in range(world + 1)]
    sizes = [3 + 2 * r for r in range(world)]
    sizes[world // 2] = 0  # a rank with no rows
    return list(np.concatenate([[0], np.cumsum(sizes)]))


def _rows(rank, bounds):
    rng = np.random.default_rng(500 + rank)
    return rng.integers(0, 256, (bounds[rank + 1] - bounds[rank]) * 48, dtype=np.uint8)


@pytest.mark.parametrize("world", [2, 3])
def test_transport_collectives_gloo(world):
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
    sent = [_blocks(r, world) for r in range(world)]
    for k, equal in enumerate((True, False)):
        bounds = _row_bounds(world, equal)
        want = np.concatenate([_rows(r, bounds) for r in range(world)]).tobytes()
        for _, _, _, gathered in res:
            assert gathered[k] == want
    for rank, rsizes, got, _ in res:
        # what each peer r sent to this rank, in rank order
        want = []
        for r in range(world):
            sizes, data = sent[r]
            off = sum(sizes[:rank]) * 32
            want.append(data[off:off + sizes[rank] * 32])
            assert rsizes[r] == sizes[rank]
        assert got == np.concatenate(want).tobytes()
