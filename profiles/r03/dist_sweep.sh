#!/bin/bash
# One-rank rehearsal of bench.py's N>1 path (--dist) on the GPU box: how much the per-step digest gather
# costs against the compute-only step, by digest-buffer depth and reserved CUs. Run from the repo root.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03_dist}
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python bench.py --no-cpu --steps 200 > $O/n1.log 2>&1
for b in 1 2 3 4; do
  timeout -k 10 120 python bench.py --dist --no-cpu --steps 200 --gather-buffers $b > $O/dist_b$b.log 2>&1
done
timeout -k 10 120 python bench.py --dist --no-cpu --steps 200 --gather-buffers 3 --reserve-cus 0 > $O/dist_b3_r0.log 2>&1
timeout -k 10 120 python bench.py --dist --no-cpu --steps 200 --gather-buffers 3 --hw-queues 4 > $O/dist_b3_q4.log 2>&1
echo sweep done
