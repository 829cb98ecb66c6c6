# coded LDS lists: routing parity tests, then C1 timings coded vs 24-B lists
set -o pipefail
D=gpurun_out/r02g
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "routing_table or c1_full or fixture or list_forms or direct or smoke" > $D/pytest.log 2>&1
rc=$?; tail -4 $D/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/routing_variants.py --c1 --reps 5 kern=slab kern=slab,coded=0 kern=slab > $D/variants.log 2>&1; rc=$?; cat $D/variants.log; exit $rc
