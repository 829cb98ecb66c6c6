# big-segment merge sort: segment parity tests, C3 bench, Zipf-destination regroup
set -o pipefail
D=gpurun_out/r02m
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -k "skewed or big_segments or oversized or medium or deliv or round or zipf or device or multirank or full_size or c3 or c4_round" > $D/pytest.log 2>&1
rc=$?; tail -6 $D/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-routing --no-cpu-baseline > $D/bench.json 2> $D/bench.err || { tail -5 $D/bench.err; exit 1; }
python -c "import json;j=json.load(open('$D/bench.json'));r=j['roofline'];print('bench', round(j['ms_per_step'],4), {k: round(v,4) for k,v in r['per_stage_ms'].items()})"
REGROUP_PIPES=slab,rank REGROUP_ZIPF=1 timeout -k 10 200 python -u scripts/bench_regroup.py > $D/regroup_zipf.log 2>&1; rc=$?; cat $D/regroup_zipf.log; [ $rc -eq 0 ] || exit $rc
REGROUP_PIPES=slab timeout -k 10 200 python -u scripts/bench_regroup.py > $D/regroup.log 2>&1; rc=$?; cat $D/regroup.log; exit $rc
