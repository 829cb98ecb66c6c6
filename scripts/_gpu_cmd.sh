set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-s6l}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
run() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-routing --no-cpu-baseline --steps 40 > gpurun_out/${T}_$tag.json 2> gpurun_out/${T}_$tag.err || { tail -20 gpurun_out/${T}_$tag.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step'],4), {k: round(v,4) for k,v in r['per_stage_ms'].items()})" gpurun_out/${T}_$tag.json $tag
}
run host SHD_SLAB_LAYOUT=host && run rankmajor SHD_SLAB_LAYOUT=rank && run host2 SHD_SLAB_LAYOUT=host && run rankmajor2 SHD_SLAB_LAYOUT=rank
