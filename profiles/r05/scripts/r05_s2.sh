# Sorted path with the wave-synchronous >= 9-line class (var_class_w8): parity first, then the config-3 line.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s2}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_var_layouts.py tests/test_gpu_sorted_edges.py > $O/pytest_sorted.log 2>&1
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python3 bench.py --config 3 --var-path sorted --no-cpu > $O/bench_c3_sorted.log 2>&1
timeout -k 10 300 python3 bench.py --config 3 --var-path sorted --no-cpu > $O/bench_c3_sorted2.log 2>&1
echo done
