#!/bin/bash
# Quick GPU check: selected GPU tests (-k expression $1) + a C1/C2/C3 bench line.
D=gpurun_out/${2:-r02q}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$1" > $D/pytest.log 2>&1
rc=$?
tail -5 $D/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --c4 0 > $D/bench.json 2> $D/bench.err || exit $?
python -c "import json;j=json.load(open('$D/bench.json'));print(j['routing']['ms_per_table'], j['routing']['c2_rows_s'], j['ms_per_step'])"
