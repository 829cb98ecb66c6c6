"""The N>1 transport on CPU: world_size-2 and 3 gloo runs of the
TorchTransport collectives exactly as libshdnet calls them (through the
ShdTransport function pointers): the count all-to-all and the contiguous
per-peer block all-to-all(v) that shd_round_exchange / _route_records issue,
and the in-place all-gather(v) of shd_topology_allgather_rows (equal blocks:
one all_gather; unequal or empty blocks: one broadcast per rank).
The GPU side (kernels, regroup, row routing) runs in test_multirank_gpu.py."""
import ctypes as C
import os
import time

import numpy as np
import pytest
import torch

from rank_procs import RankFailed, run_ranks


def _blocks(rank, world):
    """Rank's send blocks: to peer r, (rank + 1) * (r + 2) records of 32 bytes."""
    rng = np.random.default_rng(100 + rank)
    sizes = [(rank + 1) * (r + 2) for r in range(world)]
    data = rng.integers(0, 256, sum(sizes) * 32, dtype=np.uint8)
    return sizes, data


def _worker(rank, world):
    from shadow_amd.transport import TorchTransport
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
    return rank, rsizes, dst[:sum(rsizes) * 32].numpy().tobytes(), gathered


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
def test_transport_collectives_gloo(world, tmp_path):
    res = run_ranks(_worker, world, tmp_path, deadline=120)
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


def _worker_or_die(rank, world):
    return rank


@pytest.mark.timeout(90)
def test_rank_dying_before_rendezvous_fails_fast(tmp_path):
    """One rank exits before it reaches init_process_group: the harness must
    fail within seconds (not the 60 s init timeout, not a queue wait) and
    leave no live child process behind."""
    import multiprocessing
    import psutil
    before = {c.pid for c in psutil.Process().children(recursive=True)}
    t0 = time.monotonic()
    with pytest.raises(RankFailed, match="rank 1 exited with code 3"):
        run_ranks(_worker_or_die, 2, tmp_path, env={"SHD_TEST_DIE_RANK": "1"}, deadline=60)
    assert time.monotonic() - t0 < 45
    left = [c for c in psutil.Process().children(recursive=True) if c.pid not in before and c.is_running()
            and c.status() != psutil.STATUS_ZOMBIE]
    assert not left, left
    assert not [p for p in multiprocessing.active_children()]


def _worker_hang(rank, world):
    if rank == 0:
        time.sleep(600)
    return rank


@pytest.mark.timeout(90)
def test_rank_hanging_hits_the_deadline(tmp_path):
    """A rank that never reports fails the test at the parent's deadline and
    is killed, not joined forever."""
    import psutil
    before = {c.pid for c in psutil.Process().children(recursive=True)}
    t0 = time.monotonic()
    with pytest.raises(RankFailed, match="did not report"):
        run_ranks(_worker_hang, 2, tmp_path, deadline=10)
    assert time.monotonic() - t0 < 60
    left = [c for c in psutil.Process().children(recursive=True) if c.pid not in before and c.is_running()
            and c.status() != psutil.STATUS_ZOMBIE]
    assert not left, left
