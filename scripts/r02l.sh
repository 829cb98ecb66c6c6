# segment sort pass 1 by LDS broadcast: round parity tests, then C3 benches LDS=1/0 alternating
set -o pipefail
D=gpurun_out/r02l
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "round or segments or zipf or device or deliv or multirank or full_size or c3 or c4_round" > $D/pytest.log 2>&1
rc=$?; tail -4 $D/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for V in 1 0; do
    SHD_SEGSORT_LDS=$V timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-routing --no-cpu-baseline > $D/b_${V}_$i.json 2> $D/b_${V}_$i.err || { tail -5 $D/b_${V}_$i.err; exit 1; }
    python -c "import json;j=json.load(open('$D/b_${V}_$i.json'));r=j['roofline'];print('segsort_lds=$V run $i', round(j['ms_per_step'],4), {k: round(v,4) for k,v in r['per_stage_ms'].items()})"
  done
done
REGROUP_PIPES=slab REGROUP_ZIPF=1 timeout -k 10 200 python -u scripts/bench_regroup.py > $D/regroup_zipf.log 2>&1; rc=$?; cat $D/regroup_zipf.log; exit $rc
