#!/usr/bin/env python3
"""Folds rocprofv3 PMC passes into per-launch HBM traffic (bytes) per bench
stage, as MI355X_MICROARCH.md §HBM prescribes for gfx950: FETCH_SIZE counts
64 B per TCC_EA0_RDREQ while the requests are 128-B lines (x2 correction,
cross-checked against TCC_EA0_RDREQ_sum in the third pass; calibrated for
random 8..128-B gathers too -- one 128-B request each --
profiles/r04b_fetch_calibration.json); WRITE_SIZE is taken as is (it equals
64 B x WRREQ_64B + 32 B x the other write requests; a random 16-B store and a
device-scope atomic are one 32-B write request each).
Usage: scripts/traffic.py OUT.json [--suffix S] [--source TEXT] PASS_CSV...
(--suffix appends S to the routing keys and merges into an existing OUT.json,
e.g. routing_slab_c4 from a C4 build's passes)"""
import csv
import json
import re
import sys

# (a run measures one pipeline: its scatter and sort kernels name the stage;
# the record keeps the kernel, and bench.py attaches a record only to a line
# whose stage ran that kernel)
# (kernel names without their template arguments)
STAGE = {"k_pkt_scatter": "packet_scatter", "k_part_scatter": "packet_scatter", "k_part_sort": "segment_sort",
         "k_place_rank": "place", "k_place_bucket": "place", "k_segsort_dst": "segment_sort", "k_place_ovf": "place_ovf",
         "k_sssp_slab": "routing_slab", "k_sssp_islab": "routing_islab", "k_sssp_ilds": "routing_ilds",
         "k_sssp_lds": "routing_lds", "k_scan_one": "scan"}
# the path-counter fold's kernels: per fold (the add runs twice per fold, its
# small- and big-region lists: summed), folds = launches of k_fold_p1
FOLD = {"k_fold_p1": "fold_p1", "k_fold_p2": "fold_p2", "k_fold_add": "fold_add"}


def kname(n):
    m = re.search(r"(k_\w+)", n)
    return m.group(1) if m else n


def main():
    out, args = sys.argv[1], sys.argv[2:]
    suffix, source = "", None
    while args and args[0].startswith("--"):
        if args[0] == "--suffix":
            suffix, args = args[1], args[2:]
        elif args[0] == "--source":
            source, args = args[1], args[2:]
        else:
            raise SystemExit(f"unknown option {args[0]}")
    files = args
    agg = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            agg.setdefault((k, r["Counter_Name"]), []).append(float(r["Counter_Value"]))
    res = {}
    for k, st in STAGE.items():
        f, w = agg.get((k, "FETCH_SIZE")), agg.get((k, "WRITE_SIZE"))
        if not f or not w:
            continue
        rd = 2 * 1024 * sum(f) / len(f)
        wr = 1024 * sum(w) / len(w)
        rq = agg.get((k, "TCC_EA0_RDREQ_sum"))
        wq = agg.get((k, "TCC_EA0_WRREQ_sum"))
        key = st + suffix if st.startswith("routing") else st
        res[key] = {"kernel": k, "bytes": rd + wr, "read_bytes": rd, "write_bytes": wr,
                   "rd_requests": sum(rq) / len(rq) if rq else None,
                   "wr_requests": sum(wq) / len(wq) if wq else None}
    nf = len(agg.get(("k_fold_p1", "FETCH_SIZE"), []))
    for k, st in FOLD.items():
        f, w = agg.get((k, "FETCH_SIZE")), agg.get((k, "WRITE_SIZE"))
        if not f or not w or not nf:
            continue
        rq, wq = agg.get((k, "TCC_EA0_RDREQ_sum")), agg.get((k, "TCC_EA0_WRREQ_sum"))
        res[st] = {"kernel": k, "per": "fold", "folds": nf, "bytes": (2 * 1024 * sum(f) + 1024 * sum(w)) / nf,
                   "read_bytes": 2 * 1024 * sum(f) / nf, "write_bytes": 1024 * sum(w) / nf,
                   "rd_requests": sum(rq) / nf if rq else None, "wr_requests": sum(wq) / nf if wq else None}
    if suffix:
        try:
            base = json.load(open(out))
        except OSError:
            base = {}
        base.update(res)
        if source:
            base.setdefault("_sources", {})[suffix] = source
        res = base
    else:
        res["_source"] = source or ("rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE | TCC_EA0_*REQ (separate passes) over "
                                    "`bench.py --steps 3 --warmup 1 --no-routing --no-cpu-baseline`; FETCH_SIZE x2 "
                                    "(gfx950)")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
