#!/bin/bash
# SQ counters: the sorted kernel on config 3 against config 1's kernel (instructions per wave, busy/wait cycles).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-sq3}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES"
C2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_WAVES"
i=0
for C in "$C1" "$C2"; do i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'crc32_var_sorted|crc32_onekib' --output-format csv -d $O/c3s$i -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --config 3 --var-path sorted --no-cpu --steps 3 --warmup 1 > $O/c3s$i.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'crc32_onekib' --output-format csv -d $O/c1$i -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --steps 3 --warmup 1 > $O/c1$i.log 2>&1
done
for d in c3s1 c3s2 c11 c12; do f=$(find $O/$d -name '*counter_collection.csv' | head -1); python3 $GRAFT_REPO_ROOT/profiles/r05/scripts/sq_abs.py $f $d; done > $O/sq_summary.txt
rm -f $(find $O -name '*counter_collection.csv')
cat $O/sq_summary.txt
