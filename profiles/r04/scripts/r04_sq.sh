#!/bin/bash
# SQ counters (wave cycles split into parked / issue-stalled / active, instruction mixes) of the line-stream
# kernel (product and probe variants, microbench/stream_probe.py) and of the config-1 kernel for comparison.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-sq}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS"
for P in 0 7; do
  ANNETY_CRC_STREAM_PROBE=$P timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'crc32_' --output-format csv -d $O/stream_p$P -o run -- \
    python3 $GRAFT_REPO_ROOT/microbench/stream_probe.py $P > $O/stream_p$P.log 2>&1
done
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'crc32_' --output-format csv -d $O/c1 -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --prewarm-s 0.2 --steps 5 --warmup 1 > $O/c1.log 2>&1
echo done
