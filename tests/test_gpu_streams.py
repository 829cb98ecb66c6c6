"""Rounds of one topology alternating between the synchronous form (NULL
stream: the workspace's completion event recorded lazily, only when a later
use needs it) and asynchronous calls on two caller streams (recorded at
once), each with its own batch: every round must equal the same batch's
round run alone, whatever ran on the workspace before it."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_sync_and_async_rounds_interleaved():
    import torch

    from shadow_amd import Topology, scenario, synth
    H, P = 5000, 200_000
    top = Topology(synth.sparse_graph_gml(2000, 0x5EED0002))
    _, states, _ = scenario.register_hosts(top, H, seed=1)
    A = top.slot_count()
    table = top.alloc_table(A * A * 16)
    top.build_rows_device(0, A, table.ptr)
    top.adopt_table_device(table.ptr)
    top.touch_all()
    batches = [torch.from_numpy(synth.packet_batch(P - 997 * k, H, 0x5EED0E00 + k, 100_000_000, 10_000_000,
                                                   states).view(np.uint8)).cuda() for k in range(3)]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def bufs(n):
        return (torch.empty(n * 32, dtype=torch.uint8, device="cuda"), torch.empty(H + 1, dtype=torch.int32, device="cuda"),
                torch.empty(n, dtype=torch.uint8, device="cuda"), torch.empty(2, dtype=torch.int64, device="cuda"))

    def run(k, stream):
        n = batches[k].numel() // 32
        out, off, st, cnt = bufs(n)
        sp = stream.cuda_stream if stream is not None else 0
        if stream is not None:  # (the batch and the buffers were made on the default stream)
            stream.wait_stream(torch.cuda.current_stream())
        top.process_device(batches[k].data_ptr(), n, 110_000_000, 10**15, 0, out.data_ptr(), off.data_ptr(),
                           st.data_ptr(), cnt.data_ptr(), sp)
        if stream is not None:
            stream.synchronize()
        return out, off, st, cnt

    want = [run(k, None) for k in range(3)]
    torch.cuda.synchronize()
    want = [tuple(t.clone() for t in w) for w in want]
    order = [(0, s1), (1, None), (2, s2), (0, None), (1, s1), (2, None), (0, s2), (1, s2), (2, s1), (0, None)]
    for k, stream in order:
        got = run(k, stream)
        torch.cuda.synchronize()
        n = int(got[3].cpu().numpy().view(np.uint64)[0])
        assert n == int(want[k][3].cpu().numpy().view(np.uint64)[0])
        assert torch.equal(got[0][:n * 32], want[k][0][:n * 32]), (k, stream)
        for a, b in zip(got[1:], want[k][1:]):
            assert torch.equal(a, b), (k, stream)
