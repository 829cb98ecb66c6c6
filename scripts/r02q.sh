# NIC fate staging: interface/router parity tests, then the C3 bench's interface leg
set -o pipefail
D=gpurun_out/r02q
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests -m gpu -v -x --timeout 120 --timeout-method thread -k "nic or router or interfaces" > $D/pytest.log 2>&1
rc=$?; tail -4 $D/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-routing --no-cpu-baseline > $D/bench_$i.json 2> $D/bench_$i.err || { tail -5 $D/bench_$i.err; exit 1; }
python -c "import json;j=json.load(open('$D/bench_$i.json'));print('round', round(j['ms_per_step'],4), 'nic ms', round(j['nic']['ms_per_round'],4), 'received', j['nic']['received'])"
done
