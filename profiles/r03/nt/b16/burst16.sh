#!/bin/bash
# S bursts of 16 tasks (4 stores of 1 KiB per wave) with parity-split slot selects: microbench against the
# 16-task build without the parity split, GPU tests, config-3 bench lines.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-b16}
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  NO_SW=1 timeout -k 10 100 ./microbench/arena_mb > $O/amb_par_$r.log 2>&1
  NO_SW=1 timeout -k 10 100 ./microbench/arena_mb16 > $O/amb_16_$r.log 2>&1
done
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
for r in 1 2; do
  timeout -k 10 200 python bench.py --config 3 --steps 100 --warmup 10 --no-cpu > $O/c3_$r.log 2>&1
done
timeout -k 10 200 python bench.py --config 3 --var-path auto --steps 100 --warmup 10 --no-cpu > $O/c3_auto.log 2>&1
echo done
