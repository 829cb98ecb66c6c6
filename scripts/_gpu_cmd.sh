set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cp shadow_amd/libshdnet.so /tmp/libshdnet_new.so
for lib in shadow_amd/libshdnet_prev.so /tmp/libshdnet_new.so; do
  cp $lib shadow_amd/libshdnet.so
  echo "$lib"
  REGROUP_HOSTS=8000 REGROUP_PIPES=slab,slab timeout -k 10 200 python -u scripts/bench_regroup.py || exit 1
done
