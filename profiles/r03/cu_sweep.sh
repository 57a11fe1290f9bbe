#!/bin/bash
# Fewer CUs for the streaming kernels (annety_crc_reserve_cus): under the 1,400 W cap, does a smaller grid
# at a higher clock stream as fast? Configs 1 and 4, alternating reserve counts. GPU box, repo root.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/cu_sweep
mkdir -p $O
for rep in 1 2; do
  for r in 0 32 64 96; do
    timeout -k 10 60 python bench.py --config 4 --steps 40 --warmup 3 --no-cpu --reserve-cus $r > $O/c4_r${r}_$rep.log 2>&1
    timeout -k 10 60 python bench.py --steps 200 --no-cpu --reserve-cus $r > $O/c1_r${r}_$rep.log 2>&1
  done
done
