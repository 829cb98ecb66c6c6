#!/bin/bash
# GPU-box recipe (run through gpurun from the repo root):
#   scripts/gpu_run.sh TAG STEP [STEP ...]
# STEP: test[:EXPR]  pytest -m gpu (optionally -k EXPR, commas for spaces), full output in gpurun_out/TAG/
#       probe:ARGS   scripts/agg_probe.py ARGS (commas for spaces): in-process A/B of a knob
#       ubench:NAME  scripts/NAME (a microbenchmark binary built here)
#       rehearse[:ARGS]  bench.py at N=2 on one GPU over gloo (torch.distributed.run)
#       pmc          scripts/pmc_r03.sh: PMC passes over C3 rounds, C2 and C4 builds -> traffic.json
#       smoke        __graft_entry__.smoke()
#       bench[:ARGS] bench.py (ARGS: extra arguments, commas for spaces)
#       prof[:ARGS]  rocprofv3 --kernel-trace --stats of bench.py
#       run:CMD      any command (commas for spaces; may start with VAR=value
#                    assignments), output to run$i.log
# Every GPU step runs under its own time limit and the first failure ends
# the call (no further GPU work after a fault, abort or timeout).
set -o pipefail
T=$1
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=$R/gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
i=0
for step in "$@"; do
    i=$((i + 1))
    kind=${step%%:*}
    arg=""
    [[ $step == *:* ]] && arg=${step#*:}
    case $kind in
    test)
        L=$D/pytest$i.log
        if [ -n "$arg" ]; then
            timeout -k 10 1150 python -u -m pytest $R/tests -m gpu -x -v -s --durations=0 --timeout 1100 --timeout-method thread -k "${arg//,/ }" \
                > $L 2>&1 || { tail -60 $L; exit 1; }
        else
            timeout -k 10 1150 python -u -m pytest $R/tests -m gpu -x -v -s --durations=0 --timeout 1100 --timeout-method thread \
                > $L 2>&1 || { tail -60 $L; exit 1; }
        fi
        tail -3 $L ;;
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 \
            || { tail -20 $D/smoke.log; exit 1; }
        tail -1 $D/smoke.log ;;
    bench)
        timeout -k 10 900 python -u $R/bench.py ${arg//,/ } > $D/bench.json 2> $D/bench.err || { tail -30 $D/bench.err; exit 1; }
        cat $D/bench.json ;;
    probe)
        # scripts/agg_probe.py ENV V1 V2 ... (commas for spaces)
        timeout -k 10 600 python -u $R/scripts/agg_probe.py ${arg//,/ } > $D/probe$i.log 2>&1 || { tail -30 $D/probe$i.log; exit 1; }
        cat $D/probe$i.log ;;
    rehearse)
        # N=2 bench rehearsal on one GPU: both ranks on GPU 0, gloo collectives
        # (the driver's N>1 runs use RCCL over xGMI); ARGS: extra bench args
        SHD_BENCH_SHARE_GPU=1 SHD_BENCH_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 \
            --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 $R/bench.py --gpus 2 ${arg//,/ } \
            > $D/rehearse.json 2> $D/rehearse.err || { tail -30 $D/rehearse.err; exit 1; }
        cat $D/rehearse.json ;;
    ubench)
        # a prebuilt scripts/ubench_* binary (built on the CPU side with hipcc)
        timeout -k 10 300 $R/scripts/$arg > $D/$arg.log 2>&1 || { tail -20 $D/$arg.log; exit 1; }
        cat $D/$arg.log ;;
    pmc)
        timeout -k 10 1000 bash $R/scripts/pmc_r03.sh $T/pmc > $D/pmc.log 2>&1 || { tail -20 $D/pmc.log; exit 1; }
        tail -3 $D/pmc.log ;;
    prof)
        (cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -f csv -d $D/prof -o prof -- \
            python3 $R/bench.py ${arg//,/ } > $D/prof_bench.json 2> $D/prof_bench.err) || { tail -30 $D/prof_bench.err; exit 1; }
        find $D/prof -name "*kernel_stats.csv" | head -1 ;;
    run)
        timeout -k 10 900 env ${arg//,/ } > $D/run$i.log 2>&1 || { tail -30 $D/run$i.log; exit 1; }
        cat $D/run$i.log ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
done
