set -o pipefail
mkdir -p gpurun_out
T=s4o
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -k "routing or slab" --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/${T}_b.json 2>gpurun_out/${T}_b.err || { tail gpurun_out/${T}_b.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${T}_b.json'));r=d['routing'];print(round(d['ms_per_step'],4), 'C1 ms', round(r['ms_per_table'],3), 'C2 s', round(r['c2_rows_s'],3), 'C4 s', round(r['c4']['build_s'],3))"
