"""A round's fault is reported for the round that produced it (VERDICT r03
#4): with every merge wait forced to give up
(SHD_DEBUG_MERGE_SPIN=0), a round whose hot destination needs two or more
merge passes over its 4,096-event runs faults.  The faulting round itself
sets SHD_ROUND_FAULT in counters[0] (include/shdnet.h); a synchronous call
returns -EIO itself; an asynchronous call's fault is also reported once by
the next call; a clean round afterwards returns 0 and equals the oracle."""
import errno

import numpy as np
import pytest

from shadow_amd import synth
from shadow_amd._lib import ShdError
from test_gpu_parity import GRAPHS, make_pair

pytestmark = pytest.mark.gpu

ROUND_FAULT = 1 << 63
BARRIER, END = 110_000_000, 10**15


def _hot_batch(H, st):
    """90 % of 20,000 packets to host 1 (host 1's own to host 2): a segment of
    ~17k events, four 4,096-event runs and more -> merge passes 0 and 1."""
    pk = synth.packet_batch(20000, H, 0x5EED0F00, 100_000_000, 10_000_000, st)
    hot = (pk["seq"] % 10) != 0
    pk["dst_host"] = np.where(hot, np.where(pk["src_host"] == 1, 2, 1), pk["dst_host"]).astype(np.uint32)
    return pk


def _device_bufs(pk, H):
    import torch
    n = len(pk)
    return dict(recs=torch.from_numpy(pk.view(np.uint8)).cuda(),
                out=torch.empty(n * 32, dtype=torch.uint8, device="cuda"),
                off=torch.empty(H + 1, dtype=torch.int32, device="cuda"),
                status=torch.empty(n, dtype=torch.uint8, device="cuda"),
                cnt=torch.zeros(2, dtype=torch.int64, device="cuda"))


def _run(top, b, n, stream):
    top.process_device(b["recs"].data_ptr(), n, BARRIER, END, 0, b["out"].data_ptr(), b["off"].data_ptr(),
                       b["status"].data_ptr(), b["cnt"].data_ptr(), stream)


def _counters(b):
    return [int(x) for x in b["cnt"].cpu().numpy().view(np.uint64)]


@pytest.fixture
def hot_case():
    gml, H = GRAPHS["complete30_ms"]
    top, orc, ips, st = make_pair(gml, H)
    top.touch_all()
    lat, rel, sv = top.table()
    orc.preload(sv, lat, rel)
    pk = _hot_batch(H, st)
    return top, orc, ips, pk, H


def _assert_clean_round_equals_oracle(top, orc, ips, pk, H, b):
    import torch
    _run(top, b, len(pk), 0)
    torch.cuda.synchronize()
    cnt = _counters(b)
    assert not cnt[0] & ROUND_FAULT
    out = b["out"].cpu().numpy().view(synth.DELIV_DTYPE)[:cnt[0]]
    oout, ostatus, omt = orc.round(ips, pk, BARRIER, END)
    assert np.array_equal(b["status"].cpu().numpy(), ostatus) and cnt[1] == omt
    assert np.array_equal(out, oout)
    assert np.diff(b["off"].cpu().numpy()).max() > 2 * 4096  # (the merge passes ran)


def test_synchronous_round_returns_eio_for_its_own_fault(hot_case, monkeypatch):
    import torch
    top, orc, ips, pk, H = hot_case
    b = _device_bufs(pk, H)
    torch.cuda.synchronize()
    monkeypatch.setenv("SHD_DEBUG_MERGE_SPIN", "0")
    with pytest.raises(ShdError) as ei:
        _run(top, b, len(pk), 0)  # NULL stream: synchronous
    assert ei.value.code == -errno.EIO
    assert _counters(b)[0] & ROUND_FAULT
    monkeypatch.delenv("SHD_DEBUG_MERGE_SPIN")
    _assert_clean_round_equals_oracle(top, orc, ips, pk, H, b)  # reported once, not again


def test_asynchronous_round_flags_counters_then_reports_once(hot_case, monkeypatch):
    import torch
    top, orc, ips, pk, H = hot_case
    b = _device_bufs(pk, H)
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    monkeypatch.setenv("SHD_DEBUG_MERGE_SPIN", "0")
    _run(top, b, len(pk), s.cuda_stream)  # returns before the round ran
    s.synchronize()
    assert _counters(b)[0] & ROUND_FAULT  # visible with this round's own count
    monkeypatch.delenv("SHD_DEBUG_MERGE_SPIN")
    with pytest.raises(ShdError) as ei:  # the workspace's safety net: once
        _run(top, b, len(pk), s.cuda_stream)
    assert ei.value.code == -errno.EIO
    torch.cuda.synchronize()
    _assert_clean_round_equals_oracle(top, orc, ips, pk, H, b)


def test_host_api_collect_returns_eio(hot_case, monkeypatch):
    top, orc, ips, pk, H = hot_case
    monkeypatch.setenv("SHD_DEBUG_MERGE_SPIN", "0")
    with pytest.raises(ShdError) as ei:
        top.round(pk, BARRIER, END)
    assert ei.value.code == -errno.EIO
    monkeypatch.delenv("SHD_DEBUG_MERGE_SPIN")
    out, offs, status, mt = top.round(pk, BARRIER, END)
    oout, ostatus, omt = orc.round(ips, pk, BARRIER, END)
    assert np.array_equal(status, ostatus) and mt == omt and np.array_equal(out, oout)
