set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-s6h}
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-routing --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.log; exit 1; }
grep -o '"per_stage_ms": {[^}]*}' $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.log
