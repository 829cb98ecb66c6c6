set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-s6b}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
for p in slab rank; do
  SHD_PACKET_PIPELINE=$p timeout -k 10 200 python -u bench.py --no-routing --no-cpu-baseline > gpurun_out/${T}_bench_$p.json 2> gpurun_out/${T}_bench_$p.err || { tail -20 gpurun_out/${T}_bench_$p.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['ms_per_step'], r['per_stage_ms'])" gpurun_out/${T}_bench_$p.json $p
done
