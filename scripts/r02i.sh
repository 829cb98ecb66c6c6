# SQ counters over the C1 build (LDS kernel): where a pop's cycles go
D=$GRAFT_REPO_ROOT/gpurun_out/r02i
mkdir -p $D
export TMPDIR=/tmp
(cd /tmp && timeout -s KILL 60 rocprofv3 -L > $D/counters.txt 2>&1) || true
P3=""
for c in SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_SALU SQ_INSTS_SALU SQ_IFETCH; do
  grep -q "\b$c\b" $D/counters.txt && P3="$P3 $c"
done
echo "pass 3: $P3"
i=0
for GROUP in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM" \
             "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVES SQ_BUSY_CYCLES" \
             "$P3"; do
  i=$((i+1))
  [ -z "$GROUP" ] && continue
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $GROUP -f csv -d $D/p$i -o p -- python3 $GRAFT_REPO_ROOT/scripts/routing_variants.py --c1 --reps 2 kern=slab > $D/p$i.log 2>&1) || { echo "pass $i failed"; tail -5 $D/p$i.log; exit 1; }
  echo "pass $i ok"
done
