#!/bin/bash
# Config 1 with the digests stored per task (product, 0), per pair of tasks (2) and per 8 tasks (1):
# ANNETY_CRC_DIGEST_BURST, alternating, each run checks every digest against the oracle first.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/dburst
mkdir -p $O
for rep in 1 2 3; do
  for b in 0 2 1; do
    ANNETY_CRC_DIGEST_BURST=$b timeout -k 10 90 python bench.py --steps 200 --no-cpu > $O/c1_b${b}_$rep.log 2>&1
  done
done
