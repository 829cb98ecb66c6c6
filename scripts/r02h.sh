# prefetch + rotated slabs: parity tests, C1/C2/C4 routing variants, C3 rounds rot 0/1 alternating
set -o pipefail
D=gpurun_out/r02h
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "routing_table or c1_full or fixture or list_forms or slab or round or segments or zipf or device or deliv or multirank" > $D/pytest.log 2>&1
rc=$?; tail -4 $D/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/routing_variants.py --c1 --reps 5 kern=slab kern=slab,pf=1 kern=slab,coded=1,pf=1 kern=slab > $D/variants_c1.log 2>&1; rc=$?; cat $D/variants_c1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/routing_variants.py --c4 --reps 2 kern=slab kern=slab,pf=1 > $D/variants.log 2>&1; rc=$?; cat $D/variants.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for V in 0 1; do
    SHD_SLAB_ROT=$V timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-routing --no-cpu-baseline > $D/b_${V}_$i.json 2> $D/b_${V}_$i.err || { tail -5 $D/b_${V}_$i.err; exit 1; }
    python -c "import json;j=json.load(open('$D/b_${V}_$i.json'));r=j['roofline'];print('slab_rot=$V run $i', round(j['ms_per_step'],4), {k: round(v,4) for k,v in r['per_stage_ms'].items()})"
  done
done
