set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-s6e}
for b in 4 8 2 4; do
  SHD_SCATTER_BATCH=$b timeout -k 10 200 python -u bench.py --no-routing --no-cpu-baseline --steps 40 > gpurun_out/${T}_bench_b$b.json 2> gpurun_out/${T}_bench_b$b.err || { tail -20 gpurun_out/${T}_bench_b$b.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['ms_per_step'], r['per_stage_ms'])" gpurun_out/${T}_bench_b$b.json $b
done
