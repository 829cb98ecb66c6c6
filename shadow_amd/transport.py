"""Transports for multi-GPU rounds (include/shdnet.h ``ShdTransport``).

``shd_round_exchange`` / ``shd_round_route_records`` /
``shd_topology_allgather_rows`` take the collectives they need from the
caller.  Shadow's C host plugs in RCCL
(``RcclTransport``: ncclSend/ncclRecv over xGMI, inside libshdnet); these
Python transports wrap ``torch.distributed`` for tests and the benchmark:
``TorchTransport`` runs the all-to-all(v) on device tensors with the
"nccl" backend (RCCL) or bounces the blocks through host memory with "gloo".
Device buffers handed to the C calls are found among the registered tensors
(``register``) by address; anything else (the library's own scratch, e.g. the
per-destination run offsets of the exchange) is staged through a temporary
tensor with ``shd_memcpy``.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

import torch
import torch.distributed as dist

from ._lib import check, lib

A2A_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64))
A2AV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_void_p, C.POINTER(C.c_uint64),
                      C.c_void_p)
AGV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_void_p)


class ShdTransport(C.Structure):
    _fields_ = [("rank", C.c_int), ("world", C.c_int), ("user", C.c_void_p), ("alltoall_u64", A2A_FN),
                ("alltoallv", A2AV_FN), ("allgatherv", AGV_FN)]


class TorchTransport:
    def __init__(self, group=None, device=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.cdev = self.device if self.backend == "nccl" else torch.device("cpu")
        self._bufs: dict[int, torch.Tensor] = {}
        self.error: BaseException | None = None
        self._a2a = A2A_FN(self._alltoall_u64)
        self._a2av = A2AV_FN(self._alltoallv)
        self._agv = AGV_FN(self._allgatherv)
        self.struct = ShdTransport(self.rank, self.world, None, self._a2a, self._a2av, self._agv)

    def register(self, *tensors: torch.Tensor):
        """Device buffers the C calls will pass to alltoallv (by base pointer)."""
        for t in tensors:
            self._bufs[t.data_ptr()] = t.view(torch.uint8).view(-1)

    def _buf(self, ptr: int) -> torch.Tensor:
        if ptr not in self._bufs:
            raise KeyError(f"device buffer {ptr:#x} was not registered with the transport")
        return self._bufs[ptr]

    def _find(self, ptr: int, nbytes: int):
        """The registered tensor bytes [ptr, ptr + nbytes) live in, or None
        (a library-owned scratch buffer, staged through a tensor)."""
        for base, t in self._bufs.items():
            if base <= ptr and ptr + nbytes <= base + t.numel():
                return t[ptr - base:ptr - base + nbytes]
        return None

    def _stage_in(self, ptr: int, nbytes: int) -> torch.Tensor:
        v = self._find(ptr, nbytes)
        if v is not None:
            return v
        t = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=self.device)[:nbytes]
        if nbytes:
            check(lib().shd_memcpy(C.c_void_p(t.data_ptr()), C.c_void_p(ptr), nbytes))
        return t

    def _alltoall_u64(self, _user, send, recv):
        try:
            # u64 values (a failed rank sends UINT64_MAX) carried as int64 bits
            u = np.array([send[r] for r in range(self.world)], dtype=np.uint64)
            s = torch.from_numpy(u.view(np.int64)).to(self.cdev)
            out = torch.empty_like(s)
            dist.all_to_all_single(out, s, group=self.group)
            for r, v in enumerate(out.cpu().numpy().view(np.uint64).tolist()):
                recv[r] = v
            return 0
        except BaseException as e:  # never unwind through the C caller
            self.error = e
            return -5

    def _alltoallv(self, _user, d_send, send_bytes, d_recv, recv_bytes, _stream):
        try:
            sb = [int(send_bytes[r]) for r in range(self.world)]
            rb = [int(recv_bytes[r]) for r in range(self.world)]
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)  # the library's stream wrote the send side
            src = self._stage_in(d_send, sum(sb))
            dst = self._find(d_recv, sum(rb))
            staged = dst is None
            if staged:
                dst = torch.empty(max(sum(rb), 1), dtype=torch.uint8, device=self.device)[:sum(rb)]
            if self.backend == "nccl":
                dist.all_to_all_single(dst, src, rb, sb, group=self.group)
            else:
                out = torch.empty(sum(rb), dtype=torch.uint8)
                dist.all_to_all_single(out, src.cpu(), rb, sb, group=self.group)
                dst.copy_(out.to(dst.device))
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            if staged and sum(rb):
                check(lib().shd_memcpy(C.c_void_p(d_recv), C.c_void_p(dst.data_ptr()), sum(rb)))
            return 0
        except BaseException as e:
            self.error = e
            return -5

    def _allgatherv(self, _user, d_buf, offsets, _stream):
        """In place: rank r's block is bytes [offsets[r], offsets[r+1]) of the
        registered buffer d_buf; afterwards every rank holds every block."""
        try:
            off = [int(offsets[r]) for r in range(self.world + 1)]
            buf = self._buf(d_buf)[:off[-1]]
            sizes = [off[r + 1] - off[r] for r in range(self.world)]
            work = buf if self.backend == "nccl" else buf.cpu()
            if len(set(sizes)) == 1 and sizes[0]:
                mine = work[off[self.rank]:off[self.rank + 1]].clone()
                dist.all_gather_into_tensor(work, mine, group=self.group)
            else:
                for r in range(self.world):
                    if sizes[r]:
                        dist.broadcast(work[off[r]:off[r + 1]], src=r, group=self.group)
            if work is not buf:
                buf.copy_(work)
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            return 0
        except BaseException as e:
            self.error = e
            return -5

    @property
    def handle(self):
        return C.byref(self.struct)


class RcclTransport:
    """libshdnet's native RCCL transport (one communicator over the ranks of
    ``torch.distributed``'s default group, whose only role is to hand rank
    0's unique id to the others)."""

    def __init__(self, device: int):
        rank, world = dist.get_rank(), dist.get_world_size()
        uid = (C.c_char * 128)()
        if rank == 0:
            check(lib().shd_transport_rccl_unique_id(uid))
        box = [bytes(uid)]
        dist.broadcast_object_list(box, src=0)
        C.memmove(uid, box[0], 128)
        self._p = C.c_void_p()
        check(lib().shd_transport_rccl_new(rank, world, uid, device, C.byref(self._p)))
        self.rank, self.world = rank, world

    def register(self, *tensors):  # the native transport takes raw device pointers
        pass

    @property
    def handle(self):
        return self._p

    def close(self):
        if self._p:
            lib().shd_transport_rccl_free(self._p)
            self._p = C.c_void_p()


class _Rank:
    """One in-process transport (a rank that is a thread of this process)."""

    def __init__(self, handle, rank, world):
        self.handle, self.rank, self.world = handle, rank, world
        self.error = None

    def register(self, *tensors):  # (takes raw device pointers)
        pass


class InProcessTransports:
    """Transports for ranks that are threads of one process, one topology
    and one thread per device (include/shdnet.h): ``kind="local"`` --
    barrier + device-to-device copies, no RCCL (rehearsals with threads on
    one GPU); ``kind="rccl"`` -- one RCCL communicator per device from
    ncclCommInitAll (``devices`` lists them).  ``ranks[k]`` goes to the
    thread driving rank k; every rank's thread takes part in every
    collective."""

    def __init__(self, world: int, kind: str = "local", devices=None):
        arr = (C.c_void_p * world)()
        if kind == "local":
            check(lib().shd_transport_local_new(world, arr))
        else:
            devs = (C.c_int * world)(*(devices if devices is not None else range(world)))
            check(lib().shd_transport_rccl_new_all(world, devs, arr))
        self.kind = kind
        self.ranks = [_Rank(C.c_void_p(arr[k]), k, world) for k in range(world)]

    def close(self):
        for r in self.ranks:
            if r.handle and r.handle.value:
                if self.kind == "local":
                    lib().shd_transport_local_free(r.handle)
                else:
                    lib().shd_transport_rccl_free(r.handle)
                r.handle = C.c_void_p()
