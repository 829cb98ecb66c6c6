#!/usr/bin/env python3
"""Benchmark of the MI355X network plane (BASELINE.json metric:
"routed host-pairs/sec (APSP) + inter-host packets/sec per round").

`value` = inter-host packets/s per round on the C3 workload (10M synthetic
packets per round and per GPU over 100k hosts attached to the C2 sparse graph,
V=20k), whole-job aggregate over all ranks, inputs resident in HBM when the
timed region starts.  One step = one round: the packet-scatter kernel
(decision + gathers), the per-destination scan/place and the event_compare
segment sort; at N > 1 also the RCCL all-to-all of delivered events to their
destination's owner and the local regrouping there (weak scaling: 10M packets
per GPU).  The routing-table build is reported beside it ("routing": C1, the
1,000-vertex complete graph with 5,000 hosts; routed host-pairs/s = H^2 / t).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N > 1: torchrun --nproc-per-node N bench.py --gpus N ...)
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "routed host-pairs/sec (APSP) + inter-host packets/sec per round, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: 8.0 TB/s spec (6.29 measured float4 copy)
# algorithmic bytes: per packet the scatter kernel reads the
# 32 B record, 2 x 4 B host->vertex slots and the 16 B table entry and
# writes the 32 B event; place/segsort move the 32 B event in and out.
BYTES_SCATTER_PER_PKT = 32 + 2 * 4 + 16 + 32
BYTES_MOVE_PER_EVENT = 32 + 32
# path packet counters (worker.c:551): the scatter logs one u32 pair key per
# record (tables below 2^32 entries); the fold reads it back, partitions it
# and adds it into the u32 counters (PCNT_FOLD_BYTES per kept packet + the
# counter lines it touches)
PCNT_LOG_BYTES = 4
TIMING_EVERY = 4  # the timed steps whose stages carry HIP events: one in TIMING_EVERY
STAGES = ["packet_scatter", "scan", "place", "segment_sort"]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--packets", type=int, default=10_000_000, help="packets per round per GPU")
    ap.add_argument("--hosts", type=int, default=100_000)
    ap.add_argument("--vertices", type=int, default=20_000)
    ap.add_argument("--c2-hosts", type=int, default=50_000, help="C2: hosts on the V=20k graph (configs[2])")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-routing", action="store_true")
    ap.add_argument("--no-nic", action="store_true", help="skip the receive-side interface leg (§8f-2/-4)")
    ap.add_argument("--no-host-api", action="store_true", help="skip the host-API (append + collect) leg (§8b)")
    ap.add_argument("--host-workers", type=int, default=8, help="worker threads appending in the host-API leg")
    ap.add_argument("--c4", type=int, default=1, help="1: also time the C4 routing build (V=100k, H=200k)")
    ap.add_argument("--c4-vertices", type=int, default=100_000)
    ap.add_argument("--c4-hosts", type=int, default=200_000)
    ap.add_argument("--c4-rounds", type=int, default=1000, help="C4 packet rounds on the full table (N=1)")
    ap.add_argument("--c4-packets", type=int, default=1_000_000, help="packets per C4 round")
    ap.add_argument("--batches", type=int, default=4,
                    help="distinct packet batches resident in HBM, rotated so no round re-gathers the previous one's "
                         "table lines (fresh inputs per step)")
    ap.add_argument("--no-replay", action="store_true",
                    help="skip the replayed-batch comparison rounds (PMC passes: fresh rounds only)")
    ap.add_argument("--no-variants", action="store_true",
                    help="skip the §8d variant legs (ns-resolution C2 build and C3 round, C1 direct paths, Zipf C3)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "r06ai_traffic.json"),
                    help="JSON with PMC-measured HBM bytes per launch (scripts/traffic.py)")
    return ap.parse_args()


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def gpu_state(dev_index):
    """Clocks and compute/memory partition mode of the box, read from the
    amdgpu sysfs files (no subprocess: a child that re-execs under the
    profiler's preload is refused on the box), plus the device properties,
    so that run-to-run spreads can be attributed from the bench record."""
    import glob

    import torch
    p = torch.cuda.get_device_properties(dev_index)
    st = {"name": p.name, "gcn_arch": getattr(p, "gcnArchName", None), "cus": p.multi_processor_count,
          "total_mem_gb": round(p.total_memory / 2**30, 1)}
    cards = {}
    for dev in sorted(glob.glob("/sys/class/drm/card*/device")):
        info = {}
        for f in ("pp_dpm_sclk", "pp_dpm_mclk", "pp_dpm_fclk", "current_compute_partition",
                  "current_memory_partition", "power_dpm_force_performance_level"):
            try:
                with open(os.path.join(dev, f)) as fh:
                    txt = fh.read().strip()
            except OSError:
                continue
            if f.startswith("pp_dpm"):  # keep the active level (marked '*')
                txt = " ".join(ln.strip() for ln in txt.splitlines() if ln.strip().endswith("*")) or txt[:80]
            info[f] = txt
        if info:
            cards[dev.split("/")[-2]] = info
    st["sysfs"] = cards
    return st


# Random-request ceilings measured on the box by scripts/ubench_mixed.hip
# (independent random 16-B requests, by footprint and write share), the
# bound the scatter and the slab SSSP kernels are compared against beside
# their byte fraction.
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12  # 32-bit VALU lane-ops/s (MI355X_MICROARCH: 32 lanes/cycle/SIMD)
CEILING_JSON = os.path.join(ROOT, "profiles", "r04_request_ceiling.json")


def request_ceiling(key):
    try:
        with open(CEILING_JSON) as f:
            j = json.load(f)
    except OSError:
        return None, None
    return j.get(key), j.get("_source")


def request_roofline(requests, seconds, key, what):
    ceiling, src = request_ceiling(key)
    ach = requests / seconds / 1e9
    return {"bound": "random requests", "requests_per_launch": requests, "requests": what, "achieved": ach,
            "unit": "G requests/s", "peak": ceiling, "peak_case": key, "peak_source": src,
            "frac": ach / ceiling if ceiling else None}


def attainable(P, delivered, scatter_ms):
    """The scatter's attainable time: its P random 8-B table gathers at the
    measured gather ceiling, plus its streamed bytes (record 32 B + status
    1 B + counter-log key 4 B per packet, the 16-B staged event per delivered
    packet) at the HBM peak -- the two costs added, as if nothing overlapped
    them (a floor any overlap only lowers)."""
    ceiling, src = request_ceiling("gath8_3160MB")
    if not ceiling:
        return None
    g_ms = P / (ceiling * 1e9) * 1e3
    streamed = (32 + 1 + PCNT_LOG_BYTES) * P + 16.0 * delivered
    s_ms = streamed / (HBM_PEAK_GBS * 1e9) * 1e3
    return {"kernel": "k_part_scatter", "gathers": P, "gather_ceiling_G_per_s": ceiling, "gathers_ms": g_ms,
            "streamed_bytes": streamed, "streamed_ms": s_ms, "ms": g_ms + s_ms, "measured_ms": scatter_ms,
            "frac": (g_ms + s_ms) / scatter_ms, "source": src}


# The C1 kernel (k_sssp_ilds) keeps a row's whole state in LDS; its SQ
# counters (profiles/r03h_sq_c1: 640 SALU + 492 VALU + 71 LDS instructions
# per pop, one wave per SIMD, 44 % of wave cycles waiting) put it on the
# per-pop instruction chain, not on memory requests.
C1_BOUND = "salu/valu/lds instruction chain (SQ counters, profiles/r03h_sq_c1: 1,132 instr/pop, one wave per SIMD)"


# The sparse configs' latencies are whole ms, so their rows are built by the
# integer-key blocked-heap kernel; graphs with fractional-ms
# latencies use k_sssp_slab.
SLAB_KERNEL = ("k_sssp_islab (igraph-exact Dijkstra, 1 wave/source, persistent; u32 keys, 8-B heap nodes, "
               "4-level 128-B HBM blocks)")


def routing_traffic(tj, suffix):
    """PMC record of the sparse routing build (the integer-key kernel's; a
    traffic file measured on the f64 kernel has none)."""
    return tj.get("routing_islab" + suffix)


def routing_roofline(A, build_s, csr_bytes, rows, pops_per_row, traffic=None, bound="hbm (random-request rate)"):
    """Routing build roofline: compulsory bytes = the 16-B {lat, rel} table
    entries written (16 A x rows) + the CSR read once; the slab kernel is
    bound by random memory requests, so the PMC request
    count per heap pop is reported beside the byte fraction when a PMC
    record exists."""
    alg = 16.0 * A * rows + csr_bytes
    out = {"bound": bound, "alg_bytes": alg, "achieved": alg / build_s / 1e9,
           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": alg / build_s / 1e9 / HBM_PEAK_GBS,
           "pops": rows * pops_per_row}
    if traffic:
        rq = (traffic.get("rd_requests") or 0) + (traffic.get("wr_requests") or 0)
        out.update({"traffic": traffic["bytes"], "traffic_GBps": traffic["bytes"] / build_s / 1e9,
                    "requests": rq, "requests_per_pop": rq / (rows * pops_per_row) if rq else None,
                    "requests_per_s": rq / build_s if rq else None})
        if rq and bound.startswith("hbm"):
            ceil, src = request_ceiling("30720MB_37.5pct_writes")
            out["request_ceiling"] = {"peak": ceil, "unit": "G requests/s", "source": src,
                                      "frac": rq / build_s / 1e9 / ceil if ceil else None}
    return out


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from shadow_amd import Topology, _lib, scenario, synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (the driver's runs use neither): all ranks on GPU 0, and
    # gloo instead of RCCL, for checking the N>1 logic on a one-GPU box
    if os.environ.get("SHD_BENCH_SHARE_GPU") == "1":
        local = 0
    backend = os.environ.get("SHD_BENCH_BACKEND", "nccl")
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    cdev = dev if backend == "nccl" else torch.device("cpu")  # where collectives run
    stream = torch.cuda.current_stream(dev)

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    c4_ctx = None
    # ------------------------------------------------------------------ C3 setup
    H, V, P = args.hosts, args.vertices, args.packets
    t0 = time.perf_counter()
    gml = synth.sparse_graph_gml(V, 0x5EED0002)
    top = Topology(gml, device=local)
    ips, states, verts = scenario.register_hosts(top, H, seed=1)
    A = top.slot_count()
    log(f"C2 graph V={V} H={H} A={A} ready in {time.perf_counter() - t0:.1f}s")

    xport = None
    if world > 1:
        # the exchange and the all-gather run inside libshdnet
        # (shd_round_exchange, shd_topology_allgather_rows) over the library's
        # own RCCL communicator (shd_transport_rccl_new: ncclSend/ncclRecv
        # groups stream-ordered on the round's stream, the counts on the
        # transport's stream; the rank-0 unique id travels through
        # torch.distributed once).  torch.distributed's collectives
        # (TorchTransport) only for gloo rehearsals on one GPU, or SHD_XPORT=torch.
        from shadow_amd.transport import RcclTransport, TorchTransport
        use_torch = backend != "nccl" or os.environ.get("SHD_XPORT") == "torch"
        xport = TorchTransport(device=dev) if use_torch else RcclTransport(local)

    # routing rows sharded by source slot (§8e); at N>1 the full matrix the
    # replicated C3 rounds read is completed by the C-ABI all-gather
    # (shd_topology_allgather_rows over the transport's allgatherv)
    row_bounds = [min(A, r * ((A + world - 1) // world)) for r in range(world + 1)]
    lo, hi = row_bounds[rank], row_bounds[rank + 1]
    if world > 1:
        table_t = torch.empty(A * A * 2, dtype=torch.float64, device=dev)
        table_ptr = table_t.data_ptr()
        xport.register(table_t)
    else:
        table = top.alloc_table(A * A * 16)  # allocated as the library allocates its own tables
        table_ptr = table.ptr
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if hi > lo:
        top.build_rows_device(lo, hi, table_ptr)  # rows at their absolute offsets
    torch.cuda.synchronize(dev)
    t_rows_c3 = time.perf_counter() - t0
    t_ag_c3 = 0.0
    if world > 1:
        barrier()
        t0 = time.perf_counter()
        top.allgather_rows(xport, table_ptr, row_bounds, stream.cuda_stream)
        t_ag_c3 = time.perf_counter() - t0
    top.adopt_table_device(table_ptr)
    top.touch_all()  # steady state: every row released (slot order)
    log(f"C3 table {A}x{A} rows {lo}:{hi} in {t_rows_c3:.2f}s (+ all-gather {t_ag_c3:.2f}s); touched")

    # this rank's packets: senders are its src-shard hosts
    hlo, hhi = rank * H // world, (rank + 1) * H // world
    pk = synth.packet_batch(P, H, 0x5EED0003 + rank, 100_000_000, 10_000_000, states, hosts_lo=hlo, hosts_hi=hhi)
    barrier_t, end_t = 110_000_000, 10**15
    # fresh inputs per step: NB distinct batches (the same senders with new
    # destinations, synth.redraw_destinations) resident in HBM and rotated,
    # so no round gathers the table lines the previous round gathered (they
    # cannot sit in the 256 MB Infinity Cache from the step before)
    NB = max(1, args.batches)
    pks = [pk] + [synth.redraw_destinations(pk, H, 0x5EED0030 + 64 * rank + k) for k in range(1, NB)]
    d_recs_l = [torch.from_numpy(b.view(np.uint8)).to(dev) for b in pks]
    rot = {"i": 0, "fixed": None}
    d_out = torch.empty(P * 32, dtype=torch.uint8, device=dev)
    d_off = torch.empty(H + 1, dtype=torch.int32, device=dev)
    d_status = torch.empty(P, dtype=torch.uint8, device=dev)
    d_cnt = torch.empty(2, dtype=torch.int64, device=dev)
    # destination hosts owned by rank r: [own_lo[r], own_lo[r+1])
    own_lo = [r * H // world for r in range(world + 1)]
    my_lo, my_hi = own_lo[rank], own_lo[rank + 1]
    sptr = stream.cuda_stream
    last = {}
    # N>1: one call per round decides, groups by destination (unsorted),
    # ships 24-B wire records to the destinations' owners over xGMI and merges
    # them there (shd_round_process_exchange); SHD_BENCH_SPLIT=1 runs the
    # sorted round + shd_round_exchange instead
    split = os.environ.get("SHD_BENCH_SPLIT") == "1"
    if world > 1:
        wire = 32 if split else 24
        d_send = torch.empty(P * wire, dtype=torch.uint8, device=dev) if not split else d_out
        d_recv = torch.empty(2 * P * wire, dtype=torch.uint8, device=dev)
        d_final = torch.empty(2 * P * 32, dtype=torch.uint8, device=dev)
        d_final_off = torch.empty(my_hi - my_lo + 1, dtype=torch.int32, device=dev)
        xport.register(d_out, d_recv, d_send)

    # N>1: the exchange's phase times of every timed step (HIP events,
    # shd_round_exchange_phases: decide, counts, group 1, group 2, merge,
    # call, transfer beside the decide, merge beside group 2)
    xph = {"on": False, "sum": [0.0] * 8, "n": 0}
    ph_buf, ph_ok = (C.c_double * 8)(), C.c_int()

    def step():
        bi = rot["fixed"] if rot["fixed"] is not None else rot["i"] % NB
        rot["i"] += 1
        last["batch"] = bi
        d_recs = d_recs_l[bi]
        if world > 1 and not split:
            last["nrecv"] = top.process_exchange(xport, d_recs.data_ptr(), P, barrier_t, end_t, 0, own_lo,
                                                 d_send.data_ptr(), d_status.data_ptr(), d_cnt.data_ptr(),
                                                 d_recv.data_ptr(), 2 * P, d_final.data_ptr(),
                                                 d_final_off.data_ptr(), sptr)
            if xph["on"]:
                _lib.check(_lib.lib().shd_round_exchange_phases(ph_buf, 8, C.byref(ph_ok)))
                if ph_ok.value:
                    xph["sum"] = [a + b for a, b in zip(xph["sum"], ph_buf)]
                    xph["n"] += 1
            return
        top.process_device(d_recs.data_ptr(), P, barrier_t, end_t, 0, d_out.data_ptr(), d_off.data_ptr(),
                           d_status.data_ptr(), d_cnt.data_ptr(), sptr)
        if world == 1:
            return
        # destination-owner exchange (all-to-all over xGMI), then regroup
        last["nrecv"] = top.exchange(xport, d_out.data_ptr(), d_off.data_ptr(), own_lo, d_recv.data_ptr(), 2 * P,
                                     d_final.data_ptr(), d_final_off.data_ptr(), sptr)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    top.path_counts_sync()  # (the warm-up rounds' path packet counts: outside the timed region)
    state_before = gpu_state(local) if rank == 0 else None
    lib = _lib.lib()
    _lib.check(lib.shd_round_timing_enable(1))
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    xph["on"] = True
    for k in range(args.steps):
        # stage events on every TIMING_EVERY-th timed step (each event record
        # holds the next kernel back ~5 us, profiles/r05z_round_trace_gaps.log)
        _lib.check(lib.shd_round_timing_pause(int(k % TIMING_EVERY != 0)))
        step()
    xph["on"] = False
    torch.cuda.synchronize(dev)
    # topology_incrementPathPacketCounter of every kept packet (worker.c:551):
    # the rounds logged their packets' pairs; the fold that adds the K
    # rounds' logs into the counters is part of the timed work
    t_rounds = time.perf_counter()
    top.path_counts_sync()
    t_fold = time.perf_counter() - t_rounds
    barrier()
    dt = max_over_ranks(time.perf_counter() - t0)
    kept = int((d_status != 0).sum().item())  # delivered + dropped at the end time: the counted packets
    stage_ms = (C.c_double * 4)()
    nl = C.c_int()
    _lib.check(lib.shd_round_timing_read(stage_ms, 4, C.byref(nl)))
    _lib.check(lib.shd_round_timing_enable(0))
    lb = last["batch"]  # the batch of the last timed round (the legs below read its outputs)
    pk, d_recs = pks[lb], d_recs_l[lb]
    # beside it: the same K rounds replaying ONE batch (the rounds before
    # round 6 timed this form; its lines can stay cache-resident across steps)
    rep_ms = None
    if NB > 1 and not args.no_replay:
        rot["fixed"] = lb
        barrier()
        torch.cuda.synchronize(dev)
        r0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize(dev)
        top.path_counts_sync()
        barrier()
        rep_ms = max_over_ranks(time.perf_counter() - r0) / args.steps * 1e3
        rot["fixed"] = None
    cnt = d_cnt.cpu().numpy().view(np.uint64)
    delivered = int(cnt[0])
    overflow = 0
    if world == 1 or split:  # (the exchanged round keeps its offsets inside the library)
        seg = np.diff(d_off.cpu().numpy().astype(np.int64))
        overflow = int(np.maximum(seg - 256, 0).sum())  # events past their destination's 256 slab slots
    launches = max(nl.value, 1)
    per_launch_ms = [stage_ms[k] / launches for k in range(4)]
    # each rank's stage times; the roofline uses rank 0's live numbers
    dom = int(np.argmax(per_launch_ms))
    pid = C.c_int()
    _lib.check(lib.shd_round_pipeline_of(H, P, C.byref(pid)))
    pipe_name = ["bucket", "rank", "slab", "part"][pid.value]
    if pipe_name == "part":
        # k_part_scatter: record 32 B + 2 x 4 B slots + the 16 B entry (§8d) +
        # 1 B status in, the 16-B staged event out per delivered packet;
        # k_part_sort (+ listed segments): the staged event in, the 32-B event
        # and the offsets out
        kernels = ["k_part_scatter", "-", "-", "k_part_sort (+ k_segsort_mid/merge for listed segments)"]
        alg_bytes = [(32 + 2 * 4 + 16 + 1 + PCNT_LOG_BYTES) * P + 16.0 * delivered, 0.0, 0.0,
                     (16 + 32) * delivered + 4.0 * (H + 1)]
    else:
        # scan: counts in, offsets out; place: only the overflow events move
        # (k_place_ovf; 0 B when no segment outgrew its slab); sort: every
        # delivered event in and out
        kernels = ["k_pkt_scatter", "k_scan_*", "k_place_ovf", "k_segsort_dst (+ mid/merge)"]
        alg_bytes = [(BYTES_SCATTER_PER_PKT + PCNT_LOG_BYTES) * P, 4.0 * 2 * H, BYTES_MOVE_PER_EVENT * overflow,
                     BYTES_MOVE_PER_EVENT * delivered]
    achieved = [alg_bytes[k] / (per_launch_ms[k] * 1e-3) / 1e9 if per_launch_ms[k] > 0 else 0.0 for k in range(4)]
    total_pkts = P * world * args.steps
    value = total_pkts / dt
    traffic, traffic_src, tj = None, None, {}
    if args.traffic and os.path.exists(args.traffic):
        with open(args.traffic) as f:
            tj = json.load(f)
        # the PMC passes measured the default N=1 workload (10M packets, 100k
        # hosts): attached only to a line of that workload
        # and only when the record is of the kernel this line's stage ran (a
        # record without a kernel name is of the slab pipeline's kernels)
        rec = tj.get(STAGES[dom]) or {}
        want = kernels[dom].split()[0]
        have = rec.get("kernel", {"packet_scatter": "k_pkt_scatter", "segment_sort": "k_segsort_dst"}.get(STAGES[dom]))
        if rec and have == want and world == 1 and P == 10_000_000 and H == 100_000:
            traffic = tj[STAGES[dom]]["bytes"]
            traffic_src = os.path.relpath(args.traffic, ROOT) + ": " + tj.get("_source", "")

    result = {
        "metric": METRIC,
        "value": value,
        "unit": "packets/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64+f64",
        "data": "synthetic (seeded splitmix64 graph, hosts, packets; no datasets)",
        "inputs": "fresh per step" if NB > 1 else "one batch replayed every step",
        "input_batches": {"batches": NB, "rotation": "round k reads batch k mod %d (resident in HBM, %.2f GB)"
                                                       % (NB, NB * P * 32 / 1e9),
                          "what": "batch 0 = synth.packet_batch; batches 1.. = the same senders, send times and "
                                  "rand_r pre-states with new uniform destinations (synth.redraw_destinations)",
                          "fresh_ms_per_step": dt / args.steps * 1e3, "replayed_ms_per_step": rep_ms,
                          "headline": "fresh"},
        "config": {
            "workload": f"C3 per-round packet hand-off: {P / 1e6:g}M packets/round/GPU over {H / 1e3:g}k hosts on "
                        f"the C2 sparse graph (V={V / 1e3:g}k); dst-sharded with RCCL all-to-all at N>1",
            "packets_per_round_per_gpu": P, "hosts": H, "vertices": V, "attached_vertices": A,
            "delivered_per_round_rank0": delivered, "slab_overflow_events_rank0": overflow,
            "parallelism": f"dst-shard x{world}",
            "transport": None if xport is None else type(xport).__name__ + (
                " (libshdnet RCCL: ncclSend/ncclRecv)" if type(xport).__name__ == "RcclTransport"
                else f" (torch.distributed {backend})"),
        },
        "roofline": {
            "kernel": kernels[dom], "stage": STAGES[dom], "bound": "hbm", "achieved": achieved[dom],
            "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved[dom] / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
            "traffic_GBps": (traffic / (per_launch_ms[dom] * 1e-3) / 1e9) if traffic else None,
            "per_stage_ms": dict(zip(STAGES, per_launch_ms)),
            "per_stage_kernels": dict(zip(STAGES, kernels)),
            "per_stage_GBps": dict(zip(STAGES, achieved)),
            "alg_bytes_per_launch": dict(zip(STAGES, alg_bytes)),
            "timing": "HIP events on the launch stream, averaged over the timed steps that carry them "
                      "(every %d-th: an event record holds the next kernel back ~5 us)" % TIMING_EVERY,
            # the scatter's irreducible random requests: one table gather per
            # packet (3.16 GB table), against the measured rate of independent
            # 8-B gathers from a table of that size (scripts/ubench_fetch.hip)
            "request_roofline": request_roofline(float(P), per_launch_ms[0] * 1e-3, "gath8_3160MB",
                                                 "one 8-B table gather per packet (the scatter's other accesses: "
                                                 + ("streamed records, LDS staging, bucket-ordered runs"
                                                    if pipe_name == "part" else
                                                    "plus one slot atomic and one 16-B slab store per event") + ")")
            if per_launch_ms[0] > 0 else None,
            "attainable": attainable(P, delivered, per_launch_ms[0]) if pipe_name == "part" and per_launch_ms[0] > 0
            else None,
            # the whole hand-off at SURVEY.md §8d's 88 B per packet over every stage
            "handoff": {"alg_bytes_per_packet": BYTES_SCATTER_PER_PKT, "ms": sum(per_launch_ms),
                        "achieved": BYTES_SCATTER_PER_PKT * P / (sum(per_launch_ms) * 1e-3) / 1e9,
                        "frac": BYTES_SCATTER_PER_PKT * P / (sum(per_launch_ms) * 1e-3) / 1e9 / HBM_PEAK_GBS},
            "pipeline": pipe_name,
        },
        "gpu_state": {"before_timed": state_before, "after_timed": gpu_state(local) if rank == 0 else None},
        "path_counts": {
            "what": "topology_incrementPathPacketCounter of every kept packet (worker.c:551) inside the timed "
                    "region: k_part_scatter logs each record's answering pair (4 B, coalesced); at the end of "
                    "the K timed rounds shd_topology_path_counts_sync adds the K logs into the counters "
                    "(bucket partition + LDS accumulation, shd_dev_pcnt_fold; a pair's count is its u32 counter "
                    "plus its byte of the u8 delta layer the fold writes, a byte past 255 moved into the u32 "
                    "counter by the fold itself -- every count exact after the fold, no deferred merge)",
            "mode": os.environ.get("SHD_PCNT", "log"), "counted_per_round_rank0": kept,
            "fold_ms_total": t_fold * 1e3, "fold_ms_per_round": t_fold * 1e3 / args.steps,
            "rounds_per_fold": args.steps,
        },
    }

    if world > 1:
        names = ["decide", "counts", "group1", "group2", "merge", "call", "transfer_beside_decide",
                 "merge_beside_group2"]
        mine = [v / xph["n"] for v in xph["sum"]] if xph["n"] else None
        result["exchange_phases"] = {
            "what": "per timed step, HIP events on the launch and transfer streams "
                    "(shd_round_exchange_phases): decide = the sender's kernels; counts = the count-matrix "
                    "all-gather; group1 / group2 = the payload send/recv groups of owners [0, W/2) and "
                    "[W/2, W) on the transfer stream; merge = the owner merge; call = the whole "
                    "shd_round_process_exchange; transfer_beside_decide = group 1's start to the end of the "
                    "sender's kernels, merge_beside_group2 = the owner merge's time beside group 2 (the overlaps)",
            "split": mine is not None,
            "rank0_ms": dict(zip(names, mine)) if mine else None,
            "max_over_ranks_ms": dict(zip(names, [max_over_ranks(v) for v in mine])) if mine else None,
        }

    # ------------------------------------------- receive side (§8f-2 / -4)
    if not args.no_nic and world == 1:
        result["nic"] = nic_leg(lib, top, d_recs, d_out, d_off, delivered, H, dev, stream)

    # ------------------------- the drop-in host boundary at C3 size (§8b)
    if world == 1 and not args.no_host_api:
        result["host_api"] = host_api_leg(lib, top, pk, H, barrier_t, end_t, d_out, d_off, delivered,
                                          args.host_workers)

    # ------------------------------- §8d variant legs (N=1): ns, direct, Zipf
    if world == 1 and not args.no_variants:
        result["variants"] = variant_legs(args, lib, top, gml, states, pks, d_recs_l, d_out, d_off, d_status, d_cnt,
                                          dev, stream, tj)
        torch.cuda.empty_cache()

    # ------------------------------------------------------------ C1 routing
    if not args.no_routing:
        g1_v = 1000
        g1 = synth.complete_graph_gml(g1_v, 0x5EED0001)
        t1 = Topology(g1, device=local)
        scenario.register_hosts(t1, 5000, seed=1)
        A1 = t1.slot_count()
        tab1 = torch.empty(A1 * A1 * 2, dtype=torch.float64, device=dev)
        per1 = (A1 + world - 1) // world
        l1, h1 = min(A1, rank * per1), min(A1, (rank + 1) * per1)
        t1.build_rows_device(l1, h1, tab1.data_ptr())  # warm
        reps = 5
        barrier()
        torch.cuda.synchronize(dev)
        s0 = time.perf_counter()
        for _ in range(reps):
            t1.build_rows_device(l1, h1, tab1.data_ptr())
        torch.cuda.synchronize(dev)
        barrier()
        tr = max_over_ranks((time.perf_counter() - s0) / reps)
        # north_star's dense-graph kernel, latencies only (blocked min-plus
        # Floyd-Warshall; the table's reliabilities need igraph's heap order)
        fw1 = torch.empty(A1 * A1, dtype=torch.float64, device=dev)
        t1.latency_table_fw(fw1.data_ptr())  # warm
        torch.cuda.synchronize(dev)
        s0 = time.perf_counter()
        for _ in range(reps):
            t1.latency_table_fw(fw1.data_ptr())
        torch.cuda.synchronize(dev)
        t_fw1 = max_over_ranks((time.perf_counter() - s0) / reps)
        fw_vp = (g1_v + 63) // 64 * 64
        fw_same = bool(torch.equal(fw1.view(A1, A1), tab1.view(A1, A1, 2)[:, :, 0])) if world == 1 else None
        del fw1
        info1 = t1.info()
        info2 = top.info()
        t_c3 = max(max_over_ranks(t_rows_c3), 1e-9)
        result["routing"] = {
            "config": "C1 complete graph V=1000 (E=500,500 incl. self-loops), H=5000 hosts, A=%d attached" % A1,
            "value": 5000.0 ** 2 / tr, "unit": "routed host-pairs/s", "vertex_pairs_per_s": A1 * A1 / tr,
            "ms_per_table": tr * 1e3, "kernel": "k_sssp_ilds (igraph-exact Dijkstra, 1 wave/source, row in LDS, u32 keys)",
            "latency_only_minplus": {"ms": t_fw1 * 1e3, "kernel": "blocked min-plus Floyd-Warshall, 64x64 LDS tiles "
                                     "(shd_topology_latency_table_fw)", "equals_table_latencies": fw_same,
                                     # 2 Vp^3 u32 ops (one add, one min per relaxation) against the
                                     # chip's 32-bit VALU rate: 256 CUs x 4 SIMDs x 32 lanes/cycle x 2.4 GHz
                                     "valu_roofline": {"ops": 2.0 * fw_vp ** 3, "achieved": 2.0 * fw_vp ** 3 / t_fw1 / 1e12,
                                                       "peak": VALU_PEAK_TOPS, "unit": "T int32 ops/s",
                                                       "frac": 2.0 * fw_vp ** 3 / t_fw1 / 1e12 / VALU_PEAK_TOPS}},
            "roofline": routing_roofline(A1, tr, 20.0 * 2 * info1["edges"] + 4 * 1001, max(h1 - l1, 0), 1000,
                                         tj.get("routing_ilds_c1") if world == 1 else None, bound=C1_BOUND),
            "c3_table": {"config": "the C3 rounds' table: V=%d sparse graph, H=%d hosts, A=%d" % (V, H, A),
                         "rows_s": t_c3, "allgather_s": max_over_ranks(t_ag_c3) if world > 1 else 0.0,
                         "host_pairs_per_s": float(H) * H / t_c3,
                         "roofline": routing_roofline(A, t_c3, 20.0 * 2 * info2["edges"] + 4 * (V + 1),
                                                      max(hi - lo, 0), V,
                                                      routing_traffic(tj, "") if world == 1 else None)},
        }
        del tab1, t1

    # ------------------------------------------------------- C2 routing build
    # configs[2]: the V=20k sparse graph with H=50k hosts, rows sharded over
    # the ranks, the full matrix completed by the C-ABI all-gather (timed
    # separately: §8e only gathers when a full matrix is requested)
    if not args.no_routing:
        H2 = args.c2_hosts
        t2 = Topology(gml, device=local)
        scenario.register_hosts(t2, H2, seed=1)
        A2 = t2.slot_count()
        rb2 = [min(A2, r * ((A2 + world - 1) // world)) for r in range(world + 1)]
        l2, h2 = rb2[rank], rb2[rank + 1]
        tab2 = torch.empty(A2 * A2 * 2, dtype=torch.float64, device=dev)
        barrier()
        torch.cuda.synchronize(dev)
        s0 = time.perf_counter()
        if h2 > l2:
            t2.build_rows_device(l2, h2, tab2.data_ptr())
        torch.cuda.synchronize(dev)
        barrier()
        tr2 = max_over_ranks(time.perf_counter() - s0)
        tag2 = 0.0
        if world > 1:
            xport.register(tab2)
            barrier()
            s0 = time.perf_counter()
            t2.allgather_rows(xport, tab2.data_ptr(), rb2, stream.cuda_stream)
            tag2 = max_over_ranks(time.perf_counter() - s0)
        log(f"C2 V={V} H={H2} A={A2}: rows {l2}:{h2} in {tr2:.3f}s, all-gather {tag2:.3f}s")
        result["routing"]["c2"] = {
            "config": "C2 sparse graph V=%d (E=%d), H=%d hosts, A=%d attached; rows sharded over %d GPU(s)%s"
                      % (V, info2["edges"], H2, A2, world, ", full matrix all-gathered" if world > 1 else ""),
            "value": float(H2) ** 2 / tr2, "unit": "routed host-pairs/s", "vertex_pairs_per_s": float(A2) * A2 / tr2,
            "build_s": tr2, "allgather_s": tag2,
            "value_incl_allgather": float(H2) ** 2 / (tr2 + tag2),
            "kernel": SLAB_KERNEL,
            "roofline": routing_roofline(A2, tr2, 20.0 * 2 * info2["edges"] + 4 * (V + 1), max(h2 - l2, 0), V,
                                         routing_traffic(tj, "_c2") if world == 1 else None),
        }
        del tab2, t2
        torch.cuda.empty_cache()

    # ------------------------------------------------- C4 routing-table build
    # configs[4]: V=100k sparse graph, 200k hosts; rows sharded by source slot
    # across ranks (no collective: the full matrix is not requested, §8e)
    if not args.no_routing and args.c4:
        t0 = time.perf_counter()
        g4 = synth.sparse_graph_gml(args.c4_vertices, 0x5EED0004)
        t4 = Topology(g4, device=local)
        _, states4, verts4 = scenario.register_hosts(t4, args.c4_hosts, seed=1)
        c4_ctx = (g4, np.unique(verts4).astype(np.int32))  # slots = attached vertices, ascending
        A4 = t4.slot_count()
        log(f"C4 graph V={args.c4_vertices} H={args.c4_hosts} A={A4} ready in {time.perf_counter() - t0:.1f}s")
        per4 = (A4 + world - 1) // world
        l4, h4 = min(A4, rank * per4), min(A4, (rank + 1) * per4)
        shard4 = t4.alloc_table(max(h4 - l4, 1) * A4 * 16)  # allocated as the library allocates tables
        barrier()
        torch.cuda.synchronize(dev)
        s0 = time.perf_counter()
        if h4 > l4:
            # rows land at absolute offsets from the base: base = shard - l4 rows
            t4.build_rows_device(l4, h4, shard4.ptr - l4 * A4 * 16)
        torch.cuda.synchronize(dev)
        barrier()
        tr4 = max_over_ranks(time.perf_counter() - s0)
        log(f"C4 rows {l4}:{h4} of {A4} in {tr4:.2f}s")
        result.setdefault("routing", {})["c4"] = {
            "config": "C4 sparse graph V=%d, H=%d hosts, A=%d attached; rows sharded over %d GPU(s)"
                      % (args.c4_vertices, args.c4_hosts, A4, world),
            "value": float(args.c4_hosts) ** 2 / tr4, "unit": "routed host-pairs/s",
            "vertex_pairs_per_s": float(A4) * A4 / tr4, "build_s": tr4,
            "kernel": SLAB_KERNEL,
            "roofline": routing_roofline(A4, tr4, 20.0 * 2 * t4.info()["edges"] + 4 * (args.c4_vertices + 1),
                                         max(h4 - l4, 0), args.c4_vertices,
                                         routing_traffic(tj, "_c4") if world == 1 else None),
        }
        # C4 packet delivery on the 100k-vertex table as a simulation.  N=1: the
        # whole table is resident (A4^2 x 16 B = 120 GB of the 288 GB) with NO
        # row released at adoption; the first round goes through the host API
        # (shd_round_append_worker at send time: every first touch queues its
        # row's release, reduced asynchronously on the GPU; shd_round_collect
        # folds them at the boundary) -- the time to the steady state is
        # reported beside the build.  Then `c4_rounds` simulated rounds on the
        # device: the load generator (shd_synth_sends_device) has every sender
        # of the rank send m packets with its rand_r state and event counter
        # carried from round to round, new destinations every round, the
        # barrier advancing by the window.  N>1: the rows stay sharded (no full
        # matrix anywhere): each record first goes to the rank holding its
        # answering row (shd_round_route_records), is decided there, and its
        # event goes to its destination's owner (shd_round_process_exchange).
        # Weak scaling: c4_packets per rank per round.
        if args.c4_rounds > 0:
            lib4 = _lib.lib()
            P4, H4 = args.c4_packets, args.c4_hosts
            s_lo, s_hi = rank * H4 // world, (rank + 1) * H4 // world
            pool4 = np.arange(s_lo, s_hi, dtype=np.uint32)  # this rank's senders
            m4 = max(1, P4 // max(len(pool4), 1))
            n4 = len(pool4) * m4
            W4, T04, SEED4 = 10_000_000, 100_000_000, 0x5EED0008
            st4 = states4[pool4].astype(np.uint32)
            sq4 = np.zeros(len(pool4), dtype=np.uint64)
            first = None
            if world == 1:
                t4.adopt_table_device_resident(shard4.ptr)  # no 120 GB host mirror, nothing released yet
                rec0, st4, sq4 = synth.synth_sends(pool4, m4, 0, SEED4, T04, W4, st4, sq4, ndst=H4)
                nw = 8  # worker threads of the host (their buffers); appended here in worker order
                _lib.check(lib4.shd_round_set_workers(t4.handle, nw))
                _lib.check(lib4.shd_round_begin(t4.handle, T04 + W4, end_t, 0))
                bounds = [k * len(rec0) // nw for k in range(nw + 1)]
                s0 = time.perf_counter()
                for w in range(nw):
                    chunk = np.ascontiguousarray(rec0[bounds[w]:bounds[w + 1]])
                    _lib.check(lib4.shd_round_append_worker(t4.handle, w, chunk.ctypes.data, len(chunk)))
                t_app = time.perf_counter() - s0
                s0 = time.perf_counter()
                _lib.check(lib4.shd_topology_release_sync(t4.handle))
                t_rel = time.perf_counter() - s0
                seq = np.empty(A4, dtype=np.uint32)
                _lib.check(lib4.shd_topology_touch_order(t4.handle, seq.ctypes.data, None, A4))
                touched = int((seq != 0xFFFFFFFF).sum())
                out0 = np.zeros(len(rec0), dtype=synth.DELIV_DTYPE)
                offs0 = np.zeros(H4 + 1, dtype=np.uint32)
                stat0 = np.zeros(len(rec0), dtype=np.uint8)
                nout0, mt0 = C.c_size_t(), C.c_uint64()
                s0 = time.perf_counter()
                _lib.check(lib4.shd_round_collect(t4.handle, out0.ctypes.data, len(out0), C.byref(nout0),
                                                  offs0.ctypes.data, stat0.ctypes.data, C.byref(mt0)))
                t_col = time.perf_counter() - s0
                s0 = time.perf_counter()
                t4.touch_all()  # rows no host's send touched first: the steady state of the later rounds
                t_rest = time.perf_counter() - s0
                min_ms = t4.min_path_latency()
                del out0, stat0
                first = {
                    "packets": len(rec0), "senders": len(pool4), "workers": nw, "rows": A4,
                    "rows_first_touched": touched, "append_s": t_app, "release_wait_s": t_rel,
                    "collect_s": t_col, "delivered": int(nout0.value), "touch_rest_s": t_rest,
                    "steady_state_s": t_app + t_rel + t_col + t_rest,
                    "steady_state_vs_build": (t_app + t_rel + t_col + t_rest) / tr4, "min_path_latency_ms": min_ms,
                    "what": "round 0 through the host API: every host sends (shd_round_append_worker, 8 worker "
                            "buffers: the send-time lookups, first touches queue their rows' releases, launched "
                            "asynchronously in batches of 1,024); release_wait = the residual wait of the fold "
                            "(shd_topology_release_sync); collect = the round boundary incl. PCIe both ways; "
                            "touch_rest = the rows no send touched first, released in slot order",
                }
                log(f"C4 first round: {touched} of {A4} rows first-touched by the sends; append {t_app:.2f}s, "
                    f"release wait {t_rel:.3f}s, collect {t_col:.2f}s, rest {t_rest:.2f}s")
            else:
                mn = torch.tensor([t4.shard_min_latency(shard4.ptr, l4, h4) if h4 > l4 else -1.0],
                                  dtype=torch.float64, device=cdev)
                mn[mn < 0] = float("inf")
                dist.all_reduce(mn, op=dist.ReduceOp.MIN)
                t4.adopt_table_shard_device_resident(shard4.ptr, l4, h4, float(mn.item()))
            cap4 = 2 * n4
            d_pool4 = torch.from_numpy(pool4.view(np.int32)).to(dev)
            # round r reads the carried states from [r % 2] and writes [(r + 1) % 2];
            # the simulated rounds start at r = 1, so the carry starts in [1]
            d_st4 = [torch.empty(len(pool4), dtype=torch.int32, device=dev),
                     torch.from_numpy(st4.view(np.int32)).to(dev)]
            d_sq4 = [torch.empty(len(pool4), dtype=torch.int64, device=dev),
                     torch.from_numpy(sq4.view(np.int64)).to(dev)]
            r_recs = torch.empty(n4 * 32, dtype=torch.uint8, device=dev)
            r_in = torch.empty(cap4 * 32, dtype=torch.uint8, device=dev) if world > 1 else r_recs
            r_scr = torch.empty(n4 * 32, dtype=torch.uint8, device=dev) if world > 1 else None
            r_out = torch.empty(cap4 * 32, dtype=torch.uint8, device=dev)
            r_off = torch.empty(H4 + 1, dtype=torch.int32, device=dev)
            r_status = torch.empty(cap4, dtype=torch.uint8, device=dev)
            r_cnt = torch.empty(2, dtype=torch.int64, device=dev)
            row_bounds = [min(A4, r * per4) for r in range(world + 1)]
            host_bounds4 = [r * H4 // world for r in range(world + 1)]
            if world > 1:
                r_recv = torch.empty(cap4 * 32, dtype=torch.uint8, device=dev)
                r_fin = torch.empty(cap4 * 32, dtype=torch.uint8, device=dev)
                r_fin_off = torch.empty(host_bounds4[rank + 1] - host_bounds4[rank] + 1, dtype=torch.int32,
                                        device=dev)
                xport.register(r_scr, r_in, r_out, r_recv)
            rnd = [1]  # next round index (round 0 was the host-API round at N=1)

            def round4():
                r = rnd[0]
                rnd[0] += 1
                a, b = r % 2, (r + 1) % 2
                t0r = T04 + r * W4
                _lib.check(lib4.shd_synth_sends_device(
                    C.c_void_p(d_pool4.data_ptr()), len(pool4), m4, r, SEED4, t0r, W4, None, H4,
                    C.c_void_p(d_st4[a].data_ptr()), C.c_void_p(d_st4[b].data_ptr()), C.c_void_p(d_sq4[a].data_ptr()),
                    C.c_void_p(d_sq4[b].data_ptr()), C.c_void_p(r_recs.data_ptr()), C.c_void_p(sptr)))
                if world == 1:
                    t4.process_device(r_recs.data_ptr(), n4, t0r + W4, end_t, 0, r_out.data_ptr(), r_off.data_ptr(),
                                      r_status.data_ptr(), r_cnt.data_ptr(), sptr)
                    return
                # records to their answering row's rank, decided there, events to
                # their destination's owner as grouped 24-B wire records
                nr = t4.route_records(xport, r_recs.data_ptr(), n4, row_bounds, r_scr.data_ptr(),
                                      r_in.data_ptr(), cap4, sptr)
                t4.process_exchange(xport, r_in.data_ptr(), nr, t0r + W4, end_t, 0, host_bounds4, r_out.data_ptr(),
                                    r_status.data_ptr(), r_cnt.data_ptr(), r_recv.data_ptr(), cap4,
                                    r_fin.data_ptr(), r_fin_off.data_ptr(), sptr)

            for _ in range(3):
                round4()
            torch.cuda.synchronize(dev)
            t4.path_counts_sync()
            barrier()
            _lib.check(lib4.shd_round_timing_enable(1))
            s0 = time.perf_counter()
            for _ in range(args.c4_rounds):
                round4()
            torch.cuda.synchronize(dev)
            s1 = time.perf_counter()
            t4.path_counts_sync()  # the rounds' path packet counts (worker.c:551), in the timed region
            fold4 = time.perf_counter() - s1
            barrier()
            tp4 = max_over_ranks(time.perf_counter() - s0)
            # the carry reached every round: each sender's event counter advanced
            # by m per round since the state the simulated rounds started from
            sq_now = d_sq4[rnd[0] % 2].cpu().numpy().view(np.uint64)
            carry_ok = bool(np.array_equal(sq_now, sq4.astype(np.uint64) + np.uint64(m4 * (rnd[0] - 1))))
            if not carry_ok:
                raise SystemExit("C4 rounds: the carried event counters are not the expected ones")
            st4ms = (C.c_double * 4)()
            nl4 = C.c_int()
            _lib.check(lib4.shd_round_timing_read(st4ms, 4, C.byref(nl4)))
            _lib.check(lib4.shd_round_timing_enable(0))
            c4 = result["routing"]["c4"]
            if first:
                c4["first_round"] = first
            c4["rounds"] = {
                "rounds": args.c4_rounds, "packets_per_round": n4 * world, "seconds": tp4,
                "packets_per_s": n4 * world * args.c4_rounds / tp4, "ms_per_round": tp4 / args.c4_rounds * 1e3,
                "handoff_ms_per_round_rank0": sum(st4ms[k] for k in range(4)) / max(nl4.value, 1),
                "delivered_last_round_rank0": int(r_cnt.cpu().numpy().view(np.uint64)[0]),
                "carry_checked": carry_ok, "path_counts_fold_s": fold4,
                "per_round_advance": "barrier += 10 ms; every sender's rand_r state and event counter carried on the "
                                     "device; new destinations each round (shd_synth_sends_device, in the timed "
                                     "loop; handoff_ms = the decide/group/sort stages alone)",
                "input": f"each rank's {len(pool4)} senders x {m4} packets per round, destinations uniform over the "
                         f"{H4} hosts; " + ("full 120 GB table resident, rows released by round 0's sends, the "
                                            "rest in slot order" if world == 1 else
                                            "rows sharded by source slot; records routed to their answering row's "
                                            "rank, events exchanged to their destination's owner"),
            }
            log(f"C4 {args.c4_rounds} simulated rounds x {n4} packets/rank in {tp4:.2f}s")
            del r_recs, r_out, r_status
        del shard4, t4
        torch.cuda.empty_cache()

    # ------------------------------------------------------- CPU baseline (N=1)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(gml, H, states, top, result, c4_ctx, pk, args.c2_hosts)

    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        if hasattr(xport, "close"):
            xport.close()
        dist.destroy_process_group()


def timed_rounds(lib, top, recs, P, steps, warmup, dev, stream, d_out, d_off, d_status, d_cnt):
    """K device rounds (shd_round_process_device) over the resident batches
    `recs`, rotated (round k reads recs[k mod len]), timed like the headline:
    synchronize on both sides, the path-counter fold inside, HIP-event stage
    times on every TIMING_EVERY-th round.  Returns the leg's numbers and the
    scatter kernel's roofline (the same algorithmic bytes as the headline's)."""
    import torch

    from shadow_amd import _lib
    sptr = stream.cuda_stream
    it = [0]

    def one():
        top.process_device(recs[it[0] % len(recs)].data_ptr(), P, 110_000_000, 10**15, 0, d_out.data_ptr(),
                           d_off.data_ptr(), d_status.data_ptr(), d_cnt.data_ptr(), sptr)
        it[0] += 1

    for _ in range(warmup):
        one()
    torch.cuda.synchronize(dev)
    top.path_counts_sync()
    _lib.check(lib.shd_round_timing_enable(1))
    t0 = time.perf_counter()
    for k in range(steps):
        _lib.check(lib.shd_round_timing_pause(int(k % TIMING_EVERY != 0)))
        one()
    torch.cuda.synchronize(dev)
    top.path_counts_sync()
    dt = time.perf_counter() - t0
    st = (C.c_double * 4)()
    nl = C.c_int()
    _lib.check(lib.shd_round_timing_read(st, 4, C.byref(nl)))
    _lib.check(lib.shd_round_timing_enable(0))
    per = [st[k] / max(nl.value, 1) for k in range(4)]
    delivered = int(d_cnt.cpu().numpy().view(np.uint64)[0])
    alg = (32 + 2 * 4 + 16 + 1 + PCNT_LOG_BYTES) * P + 16.0 * delivered
    ach = alg / (per[0] * 1e-3) / 1e9 if per[0] > 0 else 0.0
    return {
        "rounds": steps, "batches": len(recs), "inputs": "fresh per step" if len(recs) > 1 else "one batch",
        "ms_per_step": dt / steps * 1e3, "packets_per_s": P * steps / dt, "delivered_last_round": delivered,
        "per_stage_ms": dict(zip(STAGES, per)),
        "roofline": {"kernel": "k_part_scatter", "bound": "hbm", "alg_bytes_per_launch": alg, "achieved": ach,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                     "request_roofline": request_roofline(float(P), per[0] * 1e-3, "gath8_3160MB",
                                                          "one 8-B table gather per packet") if per[0] > 0 else None,
                     "attainable": attainable(P, delivered, per[0]) if per[0] > 0 else None},
    }


def variant_legs(args, lib, top, gml, states, pks, d_recs_l, d_out, d_off, d_status, d_cnt, dev, stream, tj):
    """SURVEY.md §8d's variants beside the headline, each with its roofline
    and the CPU oracle timed on a bounded sample (cores stated):
      c2_ns_build  -- C2 (V=20k, H=50k) on the ns-resolution graph: fractional
                      ms latencies (topology.c:290-295), the f64 kernel;
      c3_ns_round  -- the C3 round on the ns-resolution graph's 100k-host table
                      (ceil(lat * 1e6) at worker.c:548 on non-integer ms);
      c1_direct    -- C1 with use_shortest_path=false: every pair's direct
                      edge (topology.c:1816-1858);
      c3_zipf      -- the C3 round with Zipf(1.1) senders (one host sends ~10%)."""
    import torch

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from shadow_amd import Topology, scenario, synth
    H, V, P = args.hosts, args.vertices, args.packets
    cpu = not args.no_cpu_baseline
    if cpu:
        import oracle_ctypes as O  # checker/baseline only
    threads = cpu_share()["threads_used"]
    out = {}
    K, W = args.steps, args.warmup
    gml_ns = synth.sparse_graph_gml(V, 0x5EED0002, ns_variant=True)

    # ---- C2 ns-variant build (f64 kernel)
    H2 = args.c2_hosts
    t2 = Topology(gml_ns, device=dev.index)
    scenario.register_hosts(t2, H2, seed=1)
    A2 = t2.slot_count()
    tab2 = torch.empty(A2 * A2 * 2, dtype=torch.float64, device=dev)
    torch.cuda.synchronize(dev)
    s0 = time.perf_counter()
    t2.build_rows_device(0, A2, tab2.data_ptr())
    torch.cuda.synchronize(dev)
    tb2 = time.perf_counter() - s0
    e2 = t2.info()["edges"]
    leg = {"config": f"C2 ns variant: V={V} sparse graph, fractional-ms latencies, H={H2} hosts, A={A2}",
           "build_s": tb2, "value": float(H2) ** 2 / tb2, "unit": "routed host-pairs/s",
           "kernel": "k_sssp_slab (igraph-exact Dijkstra, f64 keys: the latencies are not whole ms)",
           "roofline": routing_roofline(A2, tb2, 20.0 * 2 * e2 + 4 * (V + 1), A2, V, tj.get("routing_slab_c2_ns"))}
    del tab2
    if cpu:
        o2 = O.OracleTopology(gml_ns)
        _, _, v2 = scenario.register_hosts(o2, H2, seed=1)
        sv2 = np.unique(v2).astype(np.int32)
        k2 = 1024
        per = cpu_rows_parallel(o2, sv2[:: max(1, len(sv2) // k2)][:k2], sv2, threads)
        leg["cpu_baseline"] = {"value": float(H2) ** 2 / (per * len(sv2)), "unit": "routed host-pairs/s",
                               "cores": threads, "kind": "port", "build_s_extrapolated": per * len(sv2),
                               "sample": f"{k2} of {len(sv2)} source rows (evenly spaced), {threads} threads, "
                                         "extrapolated to the full table"}
        del o2
    out["c2_ns_build"] = leg
    del t2
    log(f"variant C2 ns build: {tb2:.3f}s")

    # ---- C3 round on the ns-variant table
    tn = Topology(gml_ns, device=dev.index)
    ips_n, st_n, verts_n = scenario.register_hosts(tn, H, seed=1)
    assert np.array_equal(st_n, states), "host rand_r seeds differ between the graphs"
    An = tn.slot_count()
    tabn = tn.alloc_table(An * An * 16)
    torch.cuda.synchronize(dev)
    s0 = time.perf_counter()
    tn.build_rows_device(0, An, tabn.ptr)
    torch.cuda.synchronize(dev)
    tbn = time.perf_counter() - s0
    tn.adopt_table_device(tabn.ptr)
    tn.touch_all()
    leg = timed_rounds(lib, tn, d_recs_l, P, K, W, dev, stream, d_out, d_off, d_status, d_cnt)
    leg.update({"config": f"C3 round on the ns-variant table: {P / 1e6:g}M packets over {H / 1e3:g}k hosts, "
                          f"V={V} fractional-ms graph (A={An})", "table_build_s": tbn})
    if cpu:
        n_s = 2_000_000
        pk_s = pks[0][:n_s]
        orc = O.OracleTopology(gml_ns)
        ipo, _, _ = scenario.register_hosts(orc, H, seed=1)
        lat, rel, sv = tn.table()
        orc.preload(sv, lat, rel)
        del lat, rel
        s0 = time.perf_counter()
        orc.round(ipo, pk_s, 110_000_000, 10**15)
        dtc = time.perf_counter() - s0
        leg["cpu_baseline"] = {"value": n_s / dtc, "unit": "packets/s", "cores": 1, "kind": "port",
                               "sample": f"the first {n_s} packets of batch 0 on the full ns-variant table "
                                         f"(preloaded; routing excluded): {dtc:.2f}s"}
        del orc
    out["c3_ns_round"] = leg
    del tn, tabn
    log(f"variant C3 ns round: {leg['ms_per_step']:.3f} ms")

    # ---- C1 with use_shortest_path=false (direct paths, R-10)
    g1 = synth.complete_graph_gml(1000, 0x5EED0001)
    t1 = Topology(g1, use_shortest_path=False, device=dev.index)
    _, _, v1 = scenario.register_hosts(t1, 5000, seed=1)
    A1 = t1.slot_count()
    tab1 = torch.empty(A1 * A1 * 2, dtype=torch.float64, device=dev)
    t1.build_rows_device(0, A1, tab1.data_ptr())  # warm
    reps = 10
    torch.cuda.synchronize(dev)
    s0 = time.perf_counter()
    for _ in range(reps):
        t1.build_rows_device(0, A1, tab1.data_ptr())
    torch.cuda.synchronize(dev)
    td = (time.perf_counter() - s0) / reps
    # per pair: the 16-B entry written; the edge id found in the source's
    # incidence list and the edge's weight and reliability read
    alg1 = 16.0 * A1 * A1 + 20.0 * 2 * t1.info()["edges"]
    leg = {"config": f"C1 complete graph V=1000, H=5000 hosts, A={A1}, use_shortest_path=false",
           "ms_per_table": td * 1e3, "value": 5000.0 ** 2 / td, "unit": "routed host-pairs/s",
           "kernel": "direct-path gather (shd_dev_build_rows, use_sp=0)",
           "roofline": {"bound": "hbm", "alg_bytes": alg1, "achieved": alg1 / td / 1e9, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": alg1 / td / 1e9 / HBM_PEAK_GBS}}
    if cpu:
        o1 = O.OracleTopology(g1, use_shortest_path=False)
        _, _, vo = scenario.register_hosts(o1, 5000, seed=1)
        svo = np.unique(vo).astype(np.int32)
        s0 = time.perf_counter()
        for s in svo:
            o1.direct_row(int(s), svo)
        tc = time.perf_counter() - s0
        leg["cpu_baseline"] = {"value": 5000.0 ** 2 / tc, "unit": "routed host-pairs/s", "cores": 1, "kind": "port",
                               "sample": f"all {len(svo)} rows of direct paths (orc_direct_row): {tc:.2f}s"}
        del o1
    out["c1_direct"] = leg
    del t1, tab1
    log(f"variant C1 direct: {td * 1e3:.3f} ms")

    # ---- C3 with Zipf(1.1) senders, on the headline's table
    pz = synth.packet_batch(P, H, 0x5EED0005, 100_000_000, 10_000_000, states, zipf=1.1)
    pzs = [pz] + [synth.redraw_destinations(pz, H, 0x5EED0050 + k) for k in range(1, len(d_recs_l))]
    dz = [torch.from_numpy(b.view(np.uint8)).to(dev) for b in pzs]
    leg = timed_rounds(lib, top, dz, P, K, W, dev, stream, d_out, d_off, d_status, d_cnt)
    top_share = float(np.bincount(pz["src_host"], minlength=H).max()) / P
    leg.update({"config": f"C3 with Zipf(1.1) senders: {P / 1e6:g}M packets over {H / 1e3:g}k hosts, the top "
                          f"sender {top_share:.1%} of them; destinations uniform"})
    if cpu:
        n_s = 2_000_000
        lat, rel, sv = top.table()
        orc = O.OracleTopology(gml)
        ipo, _, _ = scenario.register_hosts(orc, H, seed=1)
        orc.preload(sv, lat, rel)
        del lat, rel
        s0 = time.perf_counter()
        orc.round(ipo, pz[:n_s], 110_000_000, 10**15)
        dtc = time.perf_counter() - s0
        leg["cpu_baseline"] = {"value": n_s / dtc, "unit": "packets/s", "cores": 1, "kind": "port",
                               "sample": f"the first {n_s} packets of the Zipf batch on the full table (preloaded): "
                                         f"{dtc:.2f}s"}
        del orc
    out["c3_zipf"] = leg
    del dz
    log(f"variant C3 zipf: {leg['ms_per_step']:.3f} ms")
    return out


BYTES_NIC_PER_EVENT = 32 + 4 + 8 + 1  # event record + length in; receive time + status out
BYTES_NIC_PER_HOST = 2 * 128            # interface state read + written


def nic_leg(lib, top, d_recs, d_out, d_off, delivered, H, dev, stream, reps=5):
    """The round's delivered events, per destination segment in place, run
    through every host's interface (upstream CoDel router + receive token
    bucket + refill grid; shd_nic_run), 1 Gbit/s links, UDP headers."""
    import torch

    from shadow_amd.router import HEADER_UDP, Interfaces
    _lib_check = __import__("shadow_amd._lib", fromlist=["check"]).check
    sptr = stream.cuda_stream
    d_len = torch.empty(max(delivered, 1), dtype=torch.int32, device=dev)
    _lib_check(lib.shd_event_lengths(d_out.data_ptr(), delivered, d_recs.data_ptr(), HEADER_UDP, d_len.data_ptr(),
                                     sptr))
    times = d_out.view(torch.int64).view(-1, 4)[:delivered, 0]
    tmax = int(times.max().item()) if delivered else 0
    gbit = 1_000_000_000 // 8 // 1024  # KiB/s
    bw = np.full(H, gbit, dtype=np.uint64)
    nic = Interfaces(H, bw, bw, 100_000_000, 4096, max(delivered, 1), device=dev)
    states0 = nic.states.clone()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ms = []
    for r in range(reps + 1):
        nic.states.copy_(states0)
        torch.cuda.synchronize(dev)
        ev0.record(stream)
        nic.run_device(d_out.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), tmax + 1, 0, 0, stream=sptr)
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        if r:
            ms.append(ev0.elapsed_time(ev1))
    t = float(np.mean(ms))
    _, stat = nic.fates()
    alg = BYTES_NIC_PER_EVENT * delivered + BYTES_NIC_PER_HOST * H
    return {
        "config": "C3 round output (%d events over %d hosts), 1 Gbit/s interfaces, UDP headers, window to the last "
                  "arrival" % (delivered, H),
        "ms_per_round": t, "events_per_s": delivered / (t * 1e-3),
        "received": int((stat[:delivered] == 1).sum()), "router_dropped": int((stat[:delivered] == 2).sum()),
        "kernel": "k_nic_run (one lane per host; shd_nic_run incl. its error-word memset and read-back)",
        "roofline": {"bound": "hbm", "achieved": alg / (t * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": alg / (t * 1e-3) / 1e9 / HBM_PEAK_GBS, "alg_bytes_per_launch": alg,
                     "alg_bytes": "45 B per event (32 record + 4 length in, 8 time + 1 status out) + 256 B per host"},
    }


def host_api_leg(lib, top, pk, H, barrier_t, end_t, d_out, d_off, delivered, nworkers=8, reps=5):
    """The drop-in boundary as Shadow drives it (manager.c:553-573): during the
    round `nworkers` worker threads call shd_round_append_worker concurrently
    (each its share of the bench's C3 batch: the send-time lookups, staged in
    its own pinned buffer), then the scheduler thread calls shd_round_collect
    at the boundary (records to the device, the round -- path packet
    counters included -- and events, offsets and statuses back into pinned
    host buffers from shd_host_buffer_alloc).  Steady state: every row
    touched, buffers grown by the first (untimed) round.  The collected round
    is checked against the device round of the timed region."""
    import threading

    from shadow_amd import _lib, synth
    P = len(pk)
    h = top.handle
    _lib.check(lib.shd_round_set_workers(h, nworkers))
    bounds = [k * P // nworkers for k in range(nworkers + 1)]
    chunks = [np.ascontiguousarray(pk[bounds[w]:bounds[w + 1]]) for w in range(nworkers)]
    bufs = [C.c_void_p() for _ in range(3)]
    sizes = [P * 32, (H + 1) * 4, P]
    for b, n in zip(bufs, sizes):
        _lib.check(lib.shd_host_buffer_alloc(n, C.byref(b)))
    app, col = [], []
    nout, mt = C.c_size_t(), C.c_uint64()
    try:
        for r in range(reps + 1):
            _lib.check(lib.shd_round_begin(h, barrier_t, end_t, 0))
            gate = threading.Barrier(nworkers + 1)
            rcs = [None] * nworkers

            def work(w):
                gate.wait()
                rcs[w] = lib.shd_round_append_worker(h, w, chunks[w].ctypes.data, len(chunks[w]))
            th = [threading.Thread(target=work, args=(w,)) for w in range(nworkers)]
            for t in th:
                t.start()
            gate.wait()
            t0 = time.perf_counter()
            for t in th:
                t.join()
            t1 = time.perf_counter()
            for rc in rcs:
                _lib.check(rc)
            _lib.check(lib.shd_round_collect(h, bufs[0], P, C.byref(nout), bufs[1], bufs[2], C.byref(mt)))
            t2 = time.perf_counter()
            if r:
                app.append(t1 - t0)
                col.append(t2 - t1)
        nev = int(nout.value)
        got = np.ctypeslib.as_array(C.cast(bufs[0], C.POINTER(C.c_uint8)), shape=(nev * 32,))
        offs = np.ctypeslib.as_array(C.cast(bufs[1], C.POINTER(C.c_uint32)), shape=(H + 1,))
        same = nev == delivered and bool(np.array_equal(got, d_out[:nev * 32].cpu().numpy())) and bool(
            np.array_equal(offs.view(np.int32), d_off.cpu().numpy()))
    finally:
        for b in bufs:
            lib.shd_host_buffer_free(b)
    ta, tc = float(np.median(app)), float(np.median(col))
    moved = 32 * P + 32 * nev + 4 * (H + 1) + P
    return {
        "config": f"the bench's C3 batch ({P} packets over {H} hosts) through the drop-in host API: {nworkers} "
                  "threads append concurrently, then one collect (manager.c:553-573)",
        "value": P / (ta + tc), "unit": "packets/s", "workers": nworkers, "reps": reps,
        "append_ms": ta * 1e3, "collect_ms": tc * 1e3, "append_packets_per_s": P / ta,
        "collect_packets_per_s": P / tc, "collect_host_link_bytes": moved,
        "collect_host_link_GBps": moved / tc / 1e9,
        "equals_device_round": same,
        "what": "append = send-time lookups + staging into each worker's pinned buffer (steady state: no side "
                "effect left, one copy); collect = records H2D + the round on the device (decide, group, sort, "
                "path packet counters) + events/offsets/status D2H into pinned buffers; medians over the reps",
    }


def cpu_rows_parallel(orc, sources, targets, threads):
    """Oracle Dijkstra rows on `threads` host threads (ctypes releases the GIL
    inside orc_compute_row; rows are independent, like the reference's rows
    without its global graphLock).  Returns seconds per row, amortised."""
    from concurrent.futures import ThreadPoolExecutor
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda s: orc.row(int(s), targets), sources))
    return (time.perf_counter() - t0) / len(sources)


def cpu_share():
    """The host cores this job may use, and the evidence for the number:
    the cgroup CPU quota (/sys/fs/cgroup/cpu.max, cgroup v2; cpu.cfs_quota_us
    under v1) if one is set, the scheduler affinity, and OMP_NUM_THREADS (the
    job's CPU share as the GPU box declares it to its jobs; nproc there shows
    the whole machine).  threads = SHD_CPU_THREADS if set, else the smallest
    of the affinity and the quota, else of the affinity and the declared
    share."""
    quota, src = None, None
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(path) as f:
                txt = f.read().split()
        except OSError:
            continue
        src = f"{path}: {' '.join(txt)}"
        if path.endswith("cpu.max") and txt and txt[0] != "max" and len(txt) == 2:
            quota = int(txt[0]) / int(txt[1])
        elif path.endswith("cfs_quota_us") and txt and int(txt[0]) > 0:
            try:
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                    quota = int(txt[0]) / int(f.read().split()[0])
            except OSError:
                pass
        break
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    if os.environ.get("SHD_CPU_THREADS"):
        n, why = int(os.environ["SHD_CPU_THREADS"]), "SHD_CPU_THREADS"
    elif quota:
        n, why = max(1, min(aff, int(quota))), "min(affinity, cgroup quota)"
    elif omp and omp.isdigit() and int(omp) > 0:
        n, why = min(aff, int(omp)), "min(affinity, OMP_NUM_THREADS: the job's declared CPU share; no cgroup quota)"
    else:
        n, why = aff, "affinity (no quota, no declared share)"
    return {"threads_used": n, "threads_rule": why, "cgroup_cpu": src, "cgroup_quota_cpus": quota,
            "affinity_cpus": aff, "omp_num_threads": omp}


def host_cpu():
    """The box's CPU as the CPU baseline ran on it (model and
    core count stated): /proc/cpuinfo's model, the machine's CPUs and the
    share this job may use (cpu_share)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return dict({"cpu_model": model, "nproc": os.cpu_count()}, **cpu_share())


def cpu_baseline(gml, H, states, top, result, c4_ctx=None, pk=None, c2_hosts=50_000):
    """The oracle (C restatement of worker_sendPacket + per-destination binary
    heaps) timed on this host: the headline figure is the bench's own C3
    batch over the full table on one core; beside it the same batch on the
    job's host cores (cpu_share) and the round-2 bounded subsample."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ctypes as O  # checker/baseline only
    from shadow_amd import scenario, synth

    threads = cpu_share()["threads_used"]
    lat, rel, sv = top.table()
    base = {}
    hostinfo = host_cpu()
    if pk is not None:
        # the real C3 workload: every attached row preloaded (the GPU timed
        # region's steady state), the bench's own 10M-packet batch
        orc = O.OracleTopology(gml)
        ips, st2, verts = scenario.register_hosts(orc, H, seed=1)
        t0 = time.perf_counter()
        orc.preload(sv, lat, rel)
        t_pre = time.perf_counter() - t0
        t0 = time.perf_counter()
        out, status, mt = orc.round(ips, pk, 110_000_000, 10**15)
        dt = time.perf_counter() - t0
        base = {"value": len(pk) / dt, "unit": "packets/s", "cores": 1, "kind": "port",
                "sample": f"the bench's own C3 batch ({len(pk)} packets over {H} hosts) on the full {len(sv)}^2 "
                          f"table (preloaded in {t_pre:.1f}s, routing excluded as in the GPU timed region); "
                          f"{dt:.1f}s"}
        t0 = time.perf_counter()
        out_mt, status_mt, mt_mt = O.round_mt(orc, ips, pk, 110_000_000, 10**15, threads)
        dt_mt = time.perf_counter() - t0
        assert mt_mt == mt and len(out_mt) == len(out)
        base["handoff_mt"] = {"value": len(pk) / dt_mt, "unit": "packets/s", "cores": threads, "kind": "port",
                              "sample": f"the same C3 batch, {threads} threads sharded by source host with "
                                        f"per-destination queue mutexes; {dt_mt:.2f}s"}
        del orc, out, status, out_mt, status_mt
    # round-2 bounded subsample (1,000 rows, cache-friendly), kept for comparison
    orc = O.OracleTopology(gml)
    ips, st2, verts = scenario.register_hosts(orc, H, seed=1)
    nslot = 1000
    sub_slots = np.arange(nslot)
    sub_vert = sv[sub_slots]
    hosts = np.flatnonzero(np.isin(verts, sub_vert)).astype(np.uint32)
    orc.preload(sub_vert, lat[np.ix_(sub_slots, sub_slots)], rel[np.ix_(sub_slots, sub_slots)])
    del lat, rel
    n = 20_000_000
    pks = synth.packet_batch(n, H, 0x5EED0007, 100_000_000, 10_000_000, st2, hosts=hosts)
    t0 = time.perf_counter()
    out, status, mt = orc.round(ips, pks, 110_000_000, 10**15)
    dt = time.perf_counter() - t0
    sub = {"value": n / dt, "unit": "packets/s", "cores": 1, "kind": "port",
           "sample": f"{n} packets among the {len(hosts)} hosts attached to {nslot} of the C2 graph's attached "
                     f"vertices (a 16 MB sub-table); rows preloaded; {dt:.1f}s"}
    if not base:
        base = sub
    else:
        base["subsample_1000_rows"] = sub
    # routing baseline: oracle Dijkstra rows of C1 (1 core, the reference holds a global graphLock)
    g1 = synth.complete_graph_gml(1000, 0x5EED0001)
    o1 = O.OracleTopology(g1)
    _, _, v1 = scenario.register_hosts(o1, 5000, seed=1)
    targets = np.unique(v1).astype(np.int32)
    k = 100
    t0 = time.perf_counter()
    for s in targets[:k]:
        o1.row(int(s), targets)
    per_row = (time.perf_counter() - t0) / k
    full = per_row * len(targets)
    base["routing"] = {"value": 5000.0 ** 2 / full, "unit": "routed host-pairs/s", "cores": 1, "kind": "port",
                       "sample": f"{k} of {len(targets)} C1 source rows (igraph-0.8 Dijkstra restatement), "
                                 f"extrapolated to the full table: {full:.2f}s"}
    # row-parallel oracle on the job's host cores ("all N host
    # cores"; the count and its evidence in base["host"], cpu_share())
    per_mt = cpu_rows_parallel(o1, targets, targets, threads)
    base["routing_mt"] = {"value": 5000.0 ** 2 / (per_mt * len(targets)), "unit": "routed host-pairs/s",
                          "cores": threads, "kind": "port",
                          "sample": f"all {len(targets)} C1 source rows, {threads} threads: "
                                    f"{per_mt * len(targets):.2f}s"}
    # C2 itself (configs[2]: the V=20k graph with 50k hosts): every source
    # row on the box's CPU share, rows independent (no global graphLock)
    o2 = O.OracleTopology(gml)
    _, _, v2 = scenario.register_hosts(o2, c2_hosts, seed=1)
    sv2 = np.unique(v2).astype(np.int32)
    per2 = cpu_rows_parallel(o2, sv2, sv2, threads)
    full2 = per2 * len(sv2)
    base["routing_c2_mt"] = {"value": float(c2_hosts) ** 2 / full2, "unit": "routed host-pairs/s", "cores": threads,
                             "kind": "port",
                             "sample": f"all {len(sv2)} C2 source rows (V=20k, H={c2_hosts}), {threads} threads: "
                                       f"{full2:.2f}s", "build_s": full2}
    del o2
    if c4_ctx is not None:
        g4, sv4 = c4_ctx
        o4 = O.OracleTopology(g4)
        k4 = 512
        per4 = cpu_rows_parallel(o4, sv4[:: max(1, len(sv4) // k4)][:k4], sv4, threads)
        full4 = per4 * len(sv4)
        hosts4 = result.get("routing", {}).get("c4", {}).get("config", "")
        base["routing_c4_mt"] = {"value": None, "unit": "routed host-pairs/s", "cores": threads, "kind": "port",
                                 "sample": f"{k4} of {len(sv4)} C4 source rows (evenly spaced), {threads} threads, "
                                           f"extrapolated to the full table: {full4:.1f}s ({hosts4})",
                                 "build_s_extrapolated": full4}
        c4 = result.get("routing", {}).get("c4")
        if c4:
            base["routing_c4_mt"]["value"] = c4["value"] * c4["build_s"] / full4
    base["host"] = hostinfo
    return base


if __name__ == "__main__":
    main()
