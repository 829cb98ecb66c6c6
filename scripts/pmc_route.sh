#!/bin/bash
# SQ instruction/wait counters and HBM traffic over the C2 routing build, per
# slab-kernel variant (VARIANTS, routing_variants.py syntax; C4 too with C4=--c4)
D=$GRAFT_REPO_ROOT/gpurun_out/${1:-r02p}
mkdir -p $D
export TMPDIR=/tmp
(cd /tmp && timeout -s KILL 60 rocprofv3 -L > $D/counters.txt 2>&1) || true
grep -o "SQ_[A-Z_0-9]*" $D/counters.txt | sort -u > $D/sq_names.txt || true
i=0
for GROUP in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM" \
             "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVES SQ_BUSY_CYCLES" \
             "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $GROUP -f csv -d $D/p$i -o p -- python3 $GRAFT_REPO_ROOT/scripts/routing_variants.py --reps 1 ${C4:-} ${VARIANTS:-kern=islab kern=slab} > $D/p$i.log 2>&1) || { echo "pass $i failed"; tail -5 $D/p$i.log; exit 1; }
  echo "pass $i ok"
done
