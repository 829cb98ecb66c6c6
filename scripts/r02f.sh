# C3 rounds on the contiguous table: default slab vs SHD_SLAB_CONTIG=1, alternating processes
set -o pipefail
D=gpurun_out/r02f
mkdir -p $D
for i in 1 2; do
  for V in 0 1; do
    SHD_SLAB_CONTIG=$V timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-routing --no-cpu-baseline > $D/b_${V}_$i.json 2> $D/b_${V}_$i.err || { tail -5 $D/b_${V}_$i.err; exit 1; }
    python -c "import json;j=json.load(open('$D/b_${V}_$i.json'));r=j['roofline'];print('slab_contig=$V run $i', round(j['ms_per_step'],4), {k: round(v,4) for k,v in r['per_stage_ms'].items()})"
  done
done
