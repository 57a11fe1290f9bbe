#!/bin/bash
# PMC passes over the arena line pass, product (<0>) vs no S stores (<1>), from microbench/arena_mb; run on
# the GPU box from the repo root. One counter set per pass, each under its own time limit.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/lines_pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BIN=$GRAFT_REPO_ROOT/microbench/arena_mb
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES" \
         "TA_BUSY_avr TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "arena_lines" --output-format csv -d $OUT/p$i -o run -- $BIN > $OUT/p$i.log 2>&1
  echo "pass $i rc=$?"
done
