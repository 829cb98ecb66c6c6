#!/bin/bash
# End-of-round PMC evidence: C3 rounds (pmc), C1/C2 builds (pmcr), C4 build (pmc4); separate passes
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02z}
mkdir -p $O
export TMPDIR=/tmp
bash $R/scripts/r02_gpu.sh ${1:-r02z} pmc pmcr || exit $?
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  (cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $GROUP -f csv -d $O/pmc4/p$i -o p -- python3 $R/scripts/build_c4.py > $O/pmc4_p$i.log 2>&1) || { echo "pmc4 pass $i failed"; tail -5 $O/pmc4_p$i.log; exit 1; }
  echo "pmc4 pass $i ok: $GROUP"
done < $R/scripts/pmc_groups.txt
