#!/bin/bash
# SQ counters of the sorted path's >= 9-line class (var_class_w8: product and no-fold probe) against config 1.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-sq1}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU"
export SORTED_PROBE_CHILD=1 ANNETY_CRC_LIB=$GRAFT_REPO_ROOT/microbench/libannety_crc_ab.so ANNETY_CRC_SORTED_CLASSES=1
for P in 0 2; do
  export ANNETY_CRC_W8_PROBE=$P
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'crc32_var_sorted' --output-format csv -d $O/w8_p$P -o run -- \
    python3 $GRAFT_REPO_ROOT/microbench/sorted_probe.py > $O/w8_p$P.log 2>&1
done
unset SORTED_PROBE_CHILD ANNETY_CRC_LIB ANNETY_CRC_SORTED_CLASSES ANNETY_CRC_W8_PROBE
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'crc32_' --output-format csv -d $O/c1 -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --prewarm-s 0.2 --steps 5 --warmup 1 --sample-check > $O/c1.log 2>&1
for d in w8_p0 w8_p2 c1; do f=$(find $O/$d -name '*counter_collection.csv' | head -1); python3 $GRAFT_REPO_ROOT/profiles/r04/scripts/sq_summary.py $f $d; done > $O/sq_summary.txt
rm -f $(find $O -name '*counter_collection.csv')
cat $O/sq_summary.txt
