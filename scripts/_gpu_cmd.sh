set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-s6o}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
SHD_BENCH_BACKEND=gloo SHD_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline --no-routing > gpurun_out/${T}_bench_n2.out 2> gpurun_out/${T}_bench_n2.err || { tail -30 gpurun_out/${T}_bench_n2.err; exit 1; }
grep -o '"value": [0-9.e+]*, "unit": "packets/s"' gpurun_out/${T}_bench_n2.out
