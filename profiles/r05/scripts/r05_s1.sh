# Round-5 first pass after the cleanup (A/B switches out of the product, line-stream path removed): GPU suite,
# the driver's bench command, config 3 on the arena and sorted paths (same-box reference for this round).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s1}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1
timeout -k 10 300 python3 bench.py --config 3 --no-cpu > $O/bench_c3_arena.log 2>&1
timeout -k 10 300 python3 bench.py --config 3 --var-path sorted --no-cpu > $O/bench_c3_sorted.log 2>&1
echo done
