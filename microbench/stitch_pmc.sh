#!/bin/bash
# PMC passes over the stitch kernels of microbench/lite_mb (product stitch + lite variants); run on the GPU
# box from the repo root. One counter set per pass, each under its own time limit; stops at the first failure.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/stitch_pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BIN=$GRAFT_REPO_ROOT/microbench/lite_mb
i=0
for P in "SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex "stitch" --output-format csv -d $OUT/p$i -o run -- $BIN > $OUT/p$i.log 2>&1
  echo "pass $i rc=$?"
done
