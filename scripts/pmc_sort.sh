#!/bin/bash
# SQ counters over the C3 round's bucket sort and scatter (bench.py, C3 legs
# only): issue vs wait cycles, VALU / LDS / SALU instructions, LDS bank
# conflicts.  Usage: scripts/pmc_sort.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-sortsq}
mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU \
    SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT -f csv -d $O -o sq -- python3 $R/bench.py --steps 3 --warmup 1 \
    --no-routing --no-cpu-baseline --no-nic --c4 0 > $O/sq.log 2>&1) ||
    { echo "sort SQ pass failed"; tail -5 $O/sq.log; exit 1; }
find $O -name "*counter_collection.csv"
