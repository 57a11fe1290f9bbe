#!/bin/bash
# Half-line join through byte tables in the nontemporal kernels (configs 1, 2, 3): microbench, GPU tests,
# bench lines. A/B against the previous commit's numbers on other boxes is noisy: the microbench times the
# nibble-map kernel beside it on the same box.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-bm}
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./microbench/bytemap_mb > $O/bytemap_mb.log 2>&1
NO_SW=1 timeout -k 10 100 ./microbench/arena_mb > $O/arena_mb.log 2>&1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python bench.py --no-cpu > $O/c1.log 2>&1
timeout -k 10 200 python bench.py --config 3 --steps 100 --warmup 10 --no-cpu > $O/c3.log 2>&1
timeout -k 10 200 python bench.py --config 2 --steps 20 --warmup 3 --no-cpu > $O/c2.log 2>&1
echo done
