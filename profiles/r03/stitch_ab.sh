#!/bin/bash
# Stitch A/B (GPU box, repo root): the 512-lane two-payloads-in-flight stitch (product) against 768-lane
# blocks with one payload in flight (ANNETY_CRC_STITCH_BLK=768, 3 waves per SIMD under a 168-VGPR cap).
# Correctness of the 768 variant first, then alternating config-3 bench lines, then rocprof of each.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03_stitch}
mkdir -p $O
cd $GRAFT_REPO_ROOT
ANNETY_CRC_STITCH_BLK=768 timeout -k 10 300 python -u -m pytest tests/test_gpu_arena.py tests/test_gpu_arena_streams.py tests/test_gpu_fullsize.py tests/test_gpu_var_auto.py tests/test_lhc.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_768.log 2>&1
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --config 3 --steps 100 --warmup 10 --no-cpu --sample-check > $O/c3_512_$r.log 2>&1
  ANNETY_CRC_STITCH_BLK=768 timeout -k 10 120 python bench.py --config 3 --steps 100 --warmup 10 --no-cpu --sample-check > $O/c3_768_$r.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_512 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config 3 --steps 50 --warmup 5 --no-cpu --sample-check > $O/kt_512.log 2>&1
ANNETY_CRC_STITCH_BLK=768 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_768 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config 3 --steps 50 --warmup 5 --no-cpu --sample-check > $O/kt_768.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_auto -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config 3 --var-path auto --steps 50 --warmup 5 --no-cpu --sample-check > $O/kt_auto.log 2>&1
echo stitch ab done
