#!/bin/bash
# PMC passes (one counter group of pmc_groups.txt per rocprofv3 run, each
# under its own time limit) over a microbenchmark binary: per-kernel
# FETCH_SIZE / WRITE_SIZE / TCC_EA0 request counts for accesses of known
# count and width.  Usage: scripts/pmc_ubench.sh TAG BINARY
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
B=$R/scripts/$2
mkdir -p $O
export TMPDIR=/tmp
i=0
while read -r GROUP; do
    [ -z "$GROUP" ] && continue
    i=$((i + 1))
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $GROUP -f csv -d $O/p$i -o p -- $B > $O/p$i.log 2>&1) ||
        { echo "pass $i failed: $GROUP"; tail -5 $O/p$i.log; exit 1; }
    echo "pass $i ok: $GROUP"
done < $R/scripts/pmc_groups.txt
