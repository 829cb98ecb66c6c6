"""The per-stage round timing bench.py reports (shd_round_timing_enable /
shd_round_timing_read): HIP events on the launch stream, the part
pipeline's boundaries taken by its launches (hipExtLaunchKernel start / stop
events) or, with SHD_TM_EXT=0, by event records between launches."""
import ctypes as C
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ext", ["1", "0"], ids=["launch_events", "event_records"])
def test_stage_timing(ext, monkeypatch):
    import torch

    from shadow_amd import Topology, _lib, scenario, synth
    monkeypatch.setenv("SHD_TM_EXT", ext)
    H, P, K = 5000, 400_000, 6
    top = Topology(synth.sparse_graph_gml(2000, 0x5EED0002))
    _, states, _ = scenario.register_hosts(top, H, seed=1)
    A = top.slot_count()
    table = top.alloc_table(A * A * 16)
    top.build_rows_device(0, A, table.ptr)
    top.adopt_table_device(table.ptr)
    top.touch_all()
    pk = synth.packet_batch(P, H, 0x5EED0003, 100_000_000, 10_000_000, states)
    d_recs = torch.from_numpy(pk.view(np.uint8)).cuda()
    d_out = torch.empty(P * 32, dtype=torch.uint8, device="cuda")
    d_off = torch.empty(H + 1, dtype=torch.int32, device="cuda")
    d_status = torch.empty(P, dtype=torch.uint8, device="cuda")
    d_cnt = torch.empty(2, dtype=torch.int64, device="cuda")
    lib = _lib.lib()

    def rnd():
        top.process_device(d_recs.data_ptr(), P, 110_000_000, 10**15, 0, d_out.data_ptr(), d_off.data_ptr(),
                           d_status.data_ptr(), d_cnt.data_ptr(), 0)
    rnd()
    want = d_out.clone()
    torch.cuda.synchronize()
    _lib.check(lib.shd_round_timing_enable(1))
    t0 = time.perf_counter()
    for k in range(K + 2):  # (two more rounds with the recording paused: not counted)
        _lib.check(lib.shd_round_timing_pause(int(k >= K)))
        rnd()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    st, nl = (C.c_double * 4)(), C.c_int()
    _lib.check(lib.shd_round_timing_read(st, 4, C.byref(nl)))
    _lib.check(lib.shd_round_timing_enable(0))
    assert nl.value == K  # the paused rounds left no record
    assert st[0] > 0 and st[3] > 0, list(st)  # packet scatter, sort (the part pipeline: no scan / place)
    assert sum(st) <= wall, (list(st), wall)
    assert torch.equal(d_out, want)
