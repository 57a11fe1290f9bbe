#!/bin/bash
# Coalesced nontemporal loads in the arena line pass (config 3) and the G = 32 fixed kernel (config 2)
# against the per-line loads (ANNETY_CRC_LINES_NT=0 / ANNETY_CRC_FIXED_NT=0): GPU tests first, then bench
# lines alternating on one box.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-nt_arena}
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
for r in 1 2; do
  ANNETY_CRC_LINES_NT=0 timeout -k 10 200 python bench.py --config 3 --steps 100 --warmup 10 --no-cpu > $O/c3_line_$r.log 2>&1
  timeout -k 10 200 python bench.py --config 3 --steps 100 --warmup 10 --no-cpu > $O/c3_nt_$r.log 2>&1
  ANNETY_CRC_FIXED_NT=0 timeout -k 10 200 python bench.py --config 2 --steps 20 --warmup 3 --no-cpu > $O/c2_line_$r.log 2>&1
  timeout -k 10 200 python bench.py --config 2 --steps 20 --warmup 3 --no-cpu > $O/c2_nt_$r.log 2>&1
done
timeout -k 10 200 python bench.py --config 3 --var-path auto --steps 100 --warmup 10 --no-cpu > $O/c3_auto_nt.log 2>&1
echo done
