#!/bin/bash
# PMC passes (one rocprofv3 --pmc pass per counter group of pmc_groups.txt,
# each under its own time limit) over: the C3 rounds (bench.py, routing and
# CPU legs off), the C2 build (V=20k, H=50k) and the C4 build; folded into
# gpurun_out/TAG/traffic.json by traffic.py; plus the C1 build (x5).  Usage: scripts/pmc_r03.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r03pmc}
O=$R/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
run_passes() { # NAME LIMIT CMD...
    local name=$1 lim=$2
    shift 2
    local i=0
    while read -r GROUP; do
        [ -z "$GROUP" ] && continue
        i=$((i + 1))
        (cd /tmp && timeout -s KILL $lim rocprofv3 --pmc $GROUP -f csv -d $O/$name/p$i -o p -- "$@" > $O/${name}_p$i.log 2>&1) ||
            { echo "$name pass $i failed: $GROUP"; tail -5 $O/${name}_p$i.log; return 1; }
        echo "$name pass $i ok: $GROUP"
    done < $R/scripts/pmc_groups.txt
}
# C3_ONLY=FILE: only the C3 passes, merged into a copy of an earlier traffic.json
if [ -n "$C3_ONLY" ]; then
    cp $C3_ONLY $O/traffic.json &&
    run_passes c3 150 python3 $R/bench.py --steps 3 --warmup 1 --no-routing --no-cpu-baseline --no-nic --no-host-api --no-variants --no-replay &&
    python3 $R/scripts/traffic.py $O/traffic.json $(find $O/c3 -name "*counter_collection.csv") &&
    echo "traffic: $O/traffic.json"
    exit $?
fi
run_passes c3 150 python3 $R/bench.py --steps 3 --warmup 1 --no-routing --no-cpu-baseline --no-nic --no-host-api --no-variants --no-replay &&
run_passes c1 100 python3 $R/scripts/build_c4.py complete 1000 5000 0x5EED0001 &&
run_passes c2 150 python3 $R/scripts/build_c4.py 20000 50000 0x5EED0002 &&
run_passes c4 200 python3 $R/scripts/build_c4.py || exit 1
python3 $R/scripts/traffic.py $O/traffic.json $(find $O/c3 -name "*counter_collection.csv") > /dev/null &&
python3 $R/scripts/traffic.py $O/traffic.json --suffix _c1 --source "C1 build x5 (scripts/build_c4.py complete 1000 5000)" \
    $(find $O/c1 -name "*counter_collection.csv") > /dev/null &&
python3 $R/scripts/traffic.py $O/traffic.json --suffix _c2 --source "C2 build (scripts/build_c4.py 20000 50000)" \
    $(find $O/c2 -name "*counter_collection.csv") > /dev/null &&
python3 $R/scripts/traffic.py $O/traffic.json --suffix _c4 --source "C4 build (scripts/build_c4.py)" \
    $(find $O/c4 -name "*counter_collection.csv") && echo "traffic: $O/traffic.json"
