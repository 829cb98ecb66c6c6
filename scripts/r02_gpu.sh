#!/bin/bash
# One GPU-box session, steps chosen by name: test | bench | prof | pmc | pmcr.
#   test  pytest -m gpu (a failing assertion, exit 1, lets later steps run;
#         any other non-zero status -- timeout, abort, fault -- ends the call)
#   bench default bench line (N=1)
#   prof  rocprofv3 --kernel-trace --stats over a C3-only bench (no routing)
#   pmc   PMC passes (scripts/pmc_groups.txt) over the C3-only bench
#   pmcr  PMC passes over a routing bench (C1 + C2 builds, one C3 step)
# Usage: scripts/r02_gpu.sh TAG step [step ...]
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
ok_or_assert() { # continue on pytest's "tests failed" (1), stop on anything else
  local rc=$1
  [ $rc -eq 0 ] && return 0
  [ $rc -eq 1 ] && { echo "tests failed (continuing)"; return 0; }
  echo "step failed with status $rc: stopping"; exit $rc
}
pmc_passes() { # $1 = out dir, rest = bench args
  local D=$1; shift
  mkdir -p $D
  local i=0
  while read -r GROUP; do
    [ -z "$GROUP" ] && continue
    i=$((i+1))
    (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $GROUP -f csv -d $D/p$i -o p -- python3 $R/bench.py "$@" > $D/p$i.log 2>&1) || { echo "pmc pass $i failed: $GROUP"; tail -5 $D/p$i.log; exit 1; }
    echo "pmc pass $i ok: $GROUP"
  done < $R/scripts/pmc_groups.txt
}
for STEP in "$@"; do
  case $STEP in
    test)
      timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread --durations=15 ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest.log 2>&1
      rc=$?; tail -25 $O/pytest.log; ok_or_assert $rc ;;
    bench)
      timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
      cat $O/bench.json ;;
    prof)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o prof -- python3 $R/bench.py --steps 20 --warmup 3 --no-routing --no-cpu-baseline > $O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
      tail -1 $O/prof.log; find $O/prof -name "*kernel_stats.csv" | head -1 | xargs cut -c1-160 ;;
    pmc)
      pmc_passes $O/pmc --steps 3 --warmup 1 --no-routing --no-cpu-baseline ;;
    pmcr)
      pmc_passes $O/pmcr --steps 1 --warmup 0 --no-cpu-baseline --c4 0 ;;
    *) echo "unknown step $STEP"; exit 2 ;;
  esac
done
echo "r02_gpu done: $TAG"
