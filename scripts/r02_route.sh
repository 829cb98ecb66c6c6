#!/bin/bash
# Routing kernel check: routing parity tests, then C2 variants (LDS top 256/512)
D=gpurun_out/${1:-r02r}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "routing_table or c1_full or slab or fixture or direct or hbm" > $D/pytest.log 2>&1
rc=$?
tail -3 $D/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/routing_variants.py --reps 2 top=256 top=512 "top=512,waves=8192" > $D/variants.log 2>&1 || exit $?
cat $D/variants.log
