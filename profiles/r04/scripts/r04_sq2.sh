#!/bin/bash
# SQ counters of the sorted path's classes alone (ANNETY_CRC_SORTED_CLASSES: 1 = G = 32, 4 = small) for the
# coalesced (NT 3) and per-line (NT 0) loaders, and of config 2's crc32_fixed32_nt_kernel (the same access shape
# on fixed payloads) for comparison.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-sq2}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS"
for v in "3 1" "0 1" "3 4" "3 2"; do
  set -- $v
  PREWARM_S=0.2 REPS=5 ANNETY_CRC_SORTED_NT=$1 ANNETY_CRC_SORTED_CLASSES=$2 timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'crc32_var_sorted' --output-format csv -d $O/sorted_nt$1_c$2 -o run -- \
    python3 $GRAFT_REPO_ROOT/microbench/stream_probe.py s > $O/sorted_nt$1_c$2.log 2>&1
  python3 $GRAFT_REPO_ROOT/profiles/r04/scripts/sq_summary.py $O/sorted_nt$1_c$2/run_counter_collection.csv "nt=$1 classes=$2" >> $O/summary.txt
  rm -f $O/sorted_nt$1_c$2/run_counter_collection.csv
done
timeout -s KILL 180 rocprofv3 --pmc $C --kernel-include-regex 'crc32_fixed32' --output-format csv -d $O/c2 -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --config 2 --no-cpu --prewarm-s 0.2 --steps 3 --warmup 1 > $O/c2.log 2>&1
python3 $GRAFT_REPO_ROOT/profiles/r04/scripts/sq_summary.py $O/c2/run_counter_collection.csv "config 2" >> $O/summary.txt
rm -f $O/c2/run_counter_collection.csv
echo done
