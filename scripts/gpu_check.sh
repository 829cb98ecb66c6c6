#!/bin/bash
# One GPU-box pass: parity tests, gather microbenchmark, bench line, rocprof kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.log
if [ -x scripts/ubench_gather ] && [ "${UBENCH:-1}" = 1 ]; then
  timeout -k 10 120 ./scripts/ubench_gather > gpurun_out/${TAG}_ubench.log 2>&1 || exit 1
  cat gpurun_out/${TAG}_ubench.log
fi
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
