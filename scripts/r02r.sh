# destination aggregation + overflow wave-alloc: parity tests, in-process A/B on C3, Zipf regroup agg on/off
set -o pipefail
D=gpurun_out/r02r
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -k "skewed or big_segments or oversized or medium or deliv or round or zipf or device or multirank or full_size or c3 or c4_round" > $D/pytest.log 2>&1
rc=$?; tail -4 $D/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/agg_probe.py > $D/agg.log 2>&1; rc=$?; cat $D/agg.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
for A in 1 0; do
SHD_DEST_AGG=$A REGROUP_PIPES=slab,rank REGROUP_ZIPF=1 timeout -k 10 200 python -u scripts/bench_regroup.py > $D/regroup_zipf_$A.log 2>&1; rc=$?; echo "agg=$A"; cat $D/regroup_zipf_$A.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
done
REGROUP_PIPES=slab,rank timeout -k 10 200 python -u scripts/bench_regroup.py > $D/regroup.log 2>&1; rc=$?; cat $D/regroup.log | grep -v amdgpu.ids; exit $rc
