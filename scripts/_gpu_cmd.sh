set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-s6n}
for w in 8192 4096 6144 12288 8192; do
  SHD_SSSP_WAVES=$w timeout -k 10 200 python -u bench.py --no-routing --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/${T}_$w.json 2> gpurun_out/${T}_$w.err || { tail -20 gpurun_out/${T}_$w.err; exit 1; }
  echo "waves=$w $(grep 'C2 table' gpurun_out/${T}_$w.err)"
done
