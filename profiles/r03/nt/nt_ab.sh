#!/bin/bash
# Contiguous 1 KiB batches: crc32_onekib_nt_kernel (coalesced nontemporal loads + in-register transpose)
# against crc32_oneround_kernel<8> (ANNETY_CRC_FIXED_NT=0), GPU tests first; bench lines alternate on one box.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-nt}
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
for r in 1 2; do
  ANNETY_CRC_FIXED_NT=0 timeout -k 10 200 python bench.py --no-cpu > $O/c1_line_$r.log 2>&1
  timeout -k 10 200 python bench.py --no-cpu > $O/c1_nt_$r.log 2>&1
done
ANNETY_CRC_FIXED_NT=0 timeout -k 10 200 python bench.py --config 4 --steps 20 --warmup 3 --no-cpu > $O/c4_line.log 2>&1
timeout -k 10 200 python bench.py --config 4 --steps 20 --warmup 3 --no-cpu > $O/c4_nt.log 2>&1
echo done
