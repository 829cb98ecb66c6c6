set -o pipefail
mkdir -p gpurun_out/r02d
timeout -k 10 120 ./scripts/ubench_tlb > gpurun_out/r02d/tlb.log 2>&1; rc=$?; cat gpurun_out/r02d/tlb.log; [ $rc -eq 0 ] || exit $rc
bash scripts/r02_gpu.sh r02d pmc pmcr
