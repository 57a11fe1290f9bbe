#!/bin/bash
# SQ counters of the fused encode (frames mixed) and the sorted path on config 3.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-sq2}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES"
C2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH"
i=0
for C in "$C1" "$C2"; do i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'lhc_encode' --output-format csv -d $O/enc$i -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --config frames --op encode --no-cpu --steps 3 --warmup 1 > $O/enc$i.log 2>&1
done
for d in enc1 enc2; do f=$(find $O/$d -name '*counter_collection.csv' | head -1); python3 $GRAFT_REPO_ROOT/profiles/r05/scripts/sq_abs.py $f $d; done > $O/sq_summary.txt
rm -f $(find $O -name '*counter_collection.csv')
cat $O/sq_summary.txt
