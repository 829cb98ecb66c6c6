#!/bin/bash
# C1 (LDS kernel) variants: routing parity tests on complete graphs, then timings
D=gpurun_out/${1:-r02r1}
shift
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "routing_table or c1_full or fixture" > $D/pytest.log 2>&1
rc=$?
tail -3 $D/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/routing_variants.py --c1 --reps 5 "$@" > $D/variants.log 2>&1 || { cat $D/variants.log; exit 1; }
cat $D/variants.log
