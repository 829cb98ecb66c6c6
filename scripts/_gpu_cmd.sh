set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-s6x}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
REGROUP_HOSTS=1000 REGROUP_PIPES=slab timeout -k 10 300 python -u scripts/bench_regroup.py || exit 1
timeout -k 10 200 python -u bench.py --no-routing --no-cpu-baseline --steps 40 > gpurun_out/${T}_b.json 2> gpurun_out/${T}_b.err || { tail -20 gpurun_out/${T}_b.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(round(d['ms_per_step'],4), {k: round(v,4) for k,v in r['per_stage_ms'].items()})" gpurun_out/${T}_b.json
