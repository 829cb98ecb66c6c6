set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-s6r}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
cp shadow_amd/libshdnet.so /tmp/libshdnet_new.so
run() { # tag lib
  cp $2 shadow_amd/libshdnet.so
  timeout -k 10 200 python -u bench.py --no-routing --no-cpu-baseline --steps 40 > gpurun_out/${T}_$1.json 2> gpurun_out/${T}_$1.err || { tail -20 gpurun_out/${T}_$1.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step'],4), {k: round(v,4) for k,v in r['per_stage_ms'].items()})" gpurun_out/${T}_$1.json $1
}
run old shadow_amd/libshdnet_prev.so && run new /tmp/libshdnet_new.so && run old2 shadow_amd/libshdnet_prev.so && run new2 /tmp/libshdnet_new.so
