#!/bin/bash
# SQ counters over the C3 round's bucket sort and scatter (bench.py, C3 legs
# only), two passes: issue vs wait cycles, VALU / LDS / SALU instructions;
# then the cycles each instruction class kept the SIMD busy, vector memory
# instructions and LDS bank conflicts.  Usage: scripts/pmc_sort.sh TAG [nic]
# (nic: the interface leg runs too, for k_nic_run's counters)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-sortsq}
mkdir -p $O
export TMPDIR=/tmp
LEGS="--no-nic"
[ "$2" = nic ] && LEGS=""
i=0
for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES"; do
    i=$((i + 1))
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $G -f csv -d $O/p$i -o sq -- python3 $R/bench.py --steps 3 --warmup 1 \
        --no-routing --no-cpu-baseline $LEGS --no-host-api --c4 0 > $O/sq$i.log 2>&1) ||
        { echo "sort SQ pass $i failed"; tail -5 $O/sq$i.log; exit 1; }
done
find $O -name "*counter_collection.csv"
