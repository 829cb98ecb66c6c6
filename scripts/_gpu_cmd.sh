set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-s6s}
SHD_SSSP_COLO=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
for c in 0 1 0 1; do
  SHD_SSSP_COLO=$c timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 --c4 1 > gpurun_out/${T}_c$c.json 2> gpurun_out/${T}_c$c.err || { tail -20 gpurun_out/${T}_c$c.err; exit 1; }
  echo "colo=$c $(grep 'C2 table' gpurun_out/${T}_c$c.err) $(grep 'C4 rows' gpurun_out/${T}_c$c.err)"
done
