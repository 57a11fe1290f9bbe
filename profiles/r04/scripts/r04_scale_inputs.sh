#!/bin/bash
# Inputs for the N = 2/4/8 prediction, measured at N = 1 on one box, alternating: what the
# multi-GPU configuration costs before any gather (8 reserved CUs, 8 hardware queues), and the one-rank
# rehearsal of the distributed path with and without them. Also the sorted path's classes as separate
# launches (ANNETY_CRC_SORTED_FUSED=0) for their per-class times.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04_scale}
mkdir -p $O
cd $GRAFT_REPO_ROOT
B="python3 bench.py --steps 200 --warmup 20 --no-cpu --sample-check"
for rep in 1 2; do
  timeout -k 10 120 $B > $O/plain_$rep.log 2>&1
  timeout -k 10 120 $B --reserve-cus 8 > $O/reserve8_$rep.log 2>&1
  GPU_MAX_HW_QUEUES=8 timeout -k 10 120 $B > $O/hwq8_$rep.log 2>&1
  GPU_MAX_HW_QUEUES=8 timeout -k 10 120 $B --reserve-cus 8 > $O/hwq8_reserve8_$rep.log 2>&1
  timeout -k 10 120 $B --dist > $O/dist_$rep.log 2>&1
  timeout -k 10 120 $B --dist --reserve-cus 0 --hw-queues 4 > $O/dist_r0_q4_$rep.log 2>&1
  timeout -k 10 120 $B --config 4 > $O/c4_plain_$rep.log 2>&1
  timeout -k 10 120 $B --config 4 --dist > $O/c4_dist_$rep.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
ANNETY_CRC_SORTED_FUSED=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_sorted_unfused -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --config 3 --var-path sorted --steps 50 --warmup 5 --no-cpu > $O/kt_sorted_unfused.log 2>&1
echo "scale inputs done"
