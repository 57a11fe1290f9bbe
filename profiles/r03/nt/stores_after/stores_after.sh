#!/bin/bash
# Line pass with per-task S/SB stores issued after the next loads (linear S layout): microbench breakdown,
# GPU tests, config-3 bench (arena entry and automatic path).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-nt3}
mkdir -p $O
cd $GRAFT_REPO_ROOT
NO_SW=1 timeout -k 10 200 ./microbench/arena_mb > $O/arena_mb.log 2>&1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
for r in 1 2; do
  timeout -k 10 200 python bench.py --config 3 --steps 100 --warmup 10 --no-cpu > $O/c3_nt_$r.log 2>&1
done
timeout -k 10 200 python bench.py --config 3 --var-path auto --steps 100 --warmup 10 --no-cpu > $O/c3_auto.log 2>&1
echo done
