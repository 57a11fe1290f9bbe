#!/bin/bash
# Round-3 A/B of the store-wave arena line pass (then selected by ANNETY_CRC_LINE_SW=1; now rejected and
# moved to microbench/arena_sw.h): arena tests under it, then config-3 bench lines alternating
# with the burst line pass. Kept as the record of how profiles/r03/store_wave/ was produced.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03_sw}
mkdir -p $O
cd $GRAFT_REPO_ROOT
export ANNETY_CRC_LINE_SW=1
timeout -k 10 90 python -u -m pytest tests/test_gpu_arena.py -x -v --timeout 60 --timeout-method thread -k "golden or lengths" > $O/pytest_sw_first.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_arena.py tests/test_gpu_arena_streams.py tests/test_gpu_fullsize.py tests/test_lhc.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_sw.log 2>&1
for r in 1 2; do
  ANNETY_CRC_LINE_SW=0 timeout -k 10 120 python bench.py --config 3 --steps 100 --warmup 10 --no-cpu > $O/c3_burst_$r.log 2>&1
  ANNETY_CRC_LINE_SW=1 timeout -k 10 120 python bench.py --config 3 --steps 100 --warmup 10 --no-cpu > $O/c3_sw_$r.log 2>&1
done
unset ANNETY_CRC_LINE_SW
cd /tmp && export TMPDIR=/tmp
ANNETY_CRC_LINE_SW=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_sw -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config 3 --steps 50 --warmup 5 --no-cpu > $O/kt_sw.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt_dist -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dist --steps 50 --warmup 5 --no-cpu --prewarm-s 0.2 > $O/kt_dist.log 2>&1
echo sw ab done
