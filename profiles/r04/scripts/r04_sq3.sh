#!/bin/bash
# SQ counters of the sorted path at HEAD: the G = 32 class alone (classes 1) and the product (23).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-sq3}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS"
for v in "3 1" "3 23"; do
  set -- $v
  PREWARM_S=0.2 REPS=5 ANNETY_CRC_SORTED_NT=$1 ANNETY_CRC_SORTED_CLASSES=$2 timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'crc32_var_sorted' --output-format csv -d $O/sorted_nt$1_c$2 -o run -- \
    python3 $GRAFT_REPO_ROOT/microbench/stream_probe.py s > $O/sorted_nt$1_c$2.log 2>&1
  python3 $GRAFT_REPO_ROOT/profiles/r04/scripts/sq_summary.py $O/sorted_nt$1_c$2/run_counter_collection.csv "nt=$1 classes=$2" >> $O/summary.txt
  rm -f $O/sorted_nt$1_c$2/run_counter_collection.csv
done
echo done
