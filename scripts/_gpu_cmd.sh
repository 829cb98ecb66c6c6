set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=s5a
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
echo bench ok
R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${T}_prof -o prof -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --c4 0 > $R/gpurun_out/${T}_prof.log 2>&1) || { tail -20 gpurun_out/${T}_prof.log; exit 1; }
echo prof ok
bash scripts/pmc.sh ${T}
