#!/bin/bash
# End-of-round evidence, call A: full GPU tests, bench line, C3 rocprof, smoke, Zipf-regroup kernel stats
set -o pipefail
T=${1:-r02z}
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
bash $R/scripts/r02_gpu.sh $T test bench prof || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
(cd /tmp && REGROUP_PIPES=slab REGROUP_ZIPF=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $D/zipf -o zipf -- python3 $R/scripts/bench_regroup.py > $D/zipf.log 2>&1) || { tail -20 $D/zipf.log; exit 1; }
tail -2 $D/zipf.log
