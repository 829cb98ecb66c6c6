#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 --pmc pass per counter
# group, each under its own time limit).  Usage: scripts/pmc.sh TAG [bench args]
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
ARGS="--steps 3 --warmup 1 --no-routing --no-cpu-baseline $*"
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $GROUP -f csv -d $OUT/p$i -o p -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed: $GROUP"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok: $GROUP"
done < $GRAFT_REPO_ROOT/scripts/pmc_groups.txt
