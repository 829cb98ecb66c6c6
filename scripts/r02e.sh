# contiguous allocations: gather microbenchmark, then C2/C4 routing builds
set -o pipefail
D=gpurun_out/r02e
mkdir -p $D
timeout -k 10 150 ./scripts/ubench_tlb > $D/tlb.log 2>&1; rc=$?; cat $D/tlb.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/routing_variants.py --c4 --reps 2 kern=slab kern=slab,contig=1 kern=slab > $D/variants.log 2>&1; rc=$?; cat $D/variants.log; exit $rc
