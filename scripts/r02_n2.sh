#!/bin/bash
# N=2 rehearsal of the bench's multi-GPU path on a one-GPU box: both ranks on
# cuda:0, gloo collectives (the 8-GPU node runs the same code over RCCL).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-n2}
mkdir -p $O
export SHD_BENCH_SHARE_GPU=1 SHD_BENCH_BACKEND=gloo
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 3 --warmup 1 --packets 2000000 --c4-rounds 20 --c4-packets 200000 --no-cpu-baseline \
  > $O/bench_n2.json 2> $O/bench_n2.err || { tail -30 $O/bench_n2.err; exit 1; }
cat $O/bench_n2.json
