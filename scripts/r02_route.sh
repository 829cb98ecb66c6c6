#!/bin/bash
# Routing kernel check: routing parity tests, then C2 (+C4) kernel variants
D=gpurun_out/${1:-r02r}
shift
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "routing_table or c1_full or slab or fixture or direct or hbm or c4_sampled" > $D/pytest.log 2>&1
rc=$?
tail -5 $D/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/routing_variants.py --reps 2 "$@" > $D/variants.log 2>&1 || { cat $D/variants.log; exit 1; }
cat $D/variants.log
