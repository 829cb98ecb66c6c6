set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "round or oversized or deliv_sort or full_size or big_seg" > gpurun_out/s2f_pytest.log 2>&1 || { tail -30 gpurun_out/s2f_pytest.log; exit 1; }
tail -1 gpurun_out/s2f_pytest.log
for v in "SHD_SEGSORT=rank" "SHD_PACKET_PIPELINE=rank SHD_SEGSORT=rank"; do
  env $v timeout -k 10 200 python bench.py --no-routing --no-cpu-baseline > gpurun_out/s2f_b.json 2>/dev/null || exit 1
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/s2f_b.json'));print(round(d['ms_per_step'],4), {k:round(v,4) for k,v in d['roofline']['per_stage_ms'].items()})")"
done
