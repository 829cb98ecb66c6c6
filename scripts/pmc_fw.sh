#!/bin/bash
# SQ instruction counters over the min-plus FW on C1 (scripts/fw_probe.py):
# the VALU share of its issue cycles.  Usage: scripts/pmc_fw.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-fwsq}
mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES \
    SQ_INSTS_LDS SQ_INSTS_SALU -f csv -d $O -o fw -- python3 $R/scripts/fw_probe.py > $O/fw.log 2>&1) ||
    { echo "fw SQ pass failed"; tail -5 $O/fw.log; exit 1; }
find $O -name "*counter_collection.csv"
