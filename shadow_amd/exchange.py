"""Destination-owner exchange of delivered events between ranks.

Each rank decides the packets its own senders produced (one packet-scatter
pass over its HBM-resident batch); the delivered events come out grouped by
destination host with CSR offsets over all hosts.  Hosts are owned by ranks in
contiguous id ranges, so the events bound for rank r are one contiguous slice
[offsets[lo_r], offsets[hi_r]).  One all-to-all of the counts, then one
all-to-all(v) of the 32-byte events, hands every rank exactly its
destinations' events; the rank then regroups them (shd_deliv_sort_device)
into event_compare order.  event_compare is a total order, so the result does
not depend on the number of ranks.  With backend "nccl" this is RCCL over
xGMI; the same code runs on CPU tensors with "gloo" for tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

EVENT_BYTES = 32


def owner_bounds(nhosts: int, world: int) -> list[int]:
    """Host id ranges per rank: rank r owns [b[r], b[r+1])."""
    return [r * nhosts // world for r in range(world + 1)]


def exchange_events(events: torch.Tensor, offsets: torch.Tensor, bounds: list[int],
                    group=None) -> tuple[torch.Tensor, int, list[int]]:
    """events: uint8 tensor holding >= offsets[-1] 32-byte events grouped by
    destination; offsets: int32/int64 tensor of nhosts + 1 CSR offsets.
    Returns (received uint8 tensor, number of events received, per-source counts)."""
    world = dist.get_world_size(group)
    b = torch.tensor(bounds, dtype=torch.int64, device=offsets.device)
    cuts = offsets.to(torch.int64)[b]
    send = (cuts[1:] - cuts[:-1]).contiguous()
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    sc = send.cpu().tolist()
    rc = recv.cpu().tolist()
    assert len(sc) == world
    nrecv = int(sum(rc))
    nsend = int(sum(sc))
    out = torch.empty(max(nrecv, 1) * EVENT_BYTES, dtype=torch.uint8, device=events.device)
    dist.all_to_all_single(out[:nrecv * EVENT_BYTES], events[:nsend * EVENT_BYTES].contiguous(),
                           [c * EVENT_BYTES for c in rc], [c * EVENT_BYTES for c in sc], group=group)
    return out, nrecv, rc
