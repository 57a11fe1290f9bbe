# Sorted path (w8 with task-ahead descriptors, s8 small class) + fused encode: parity, probes, frames lines.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s4}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_var_layouts.py tests/test_gpu_sorted_edges.py tests/test_lhc.py -m gpu > $O/pytest_sorted_lhc.log 2>&1
timeout -k 10 500 python3 microbench/sorted_probe.py 3:0 1:0 2:0 3:1 3:2 > $O/sorted_probe.log 2>&1
timeout -k 10 300 python3 bench.py --config 3 --var-path sorted --no-cpu > $O/bench_c3_sorted.log 2>&1
timeout -k 10 300 python3 bench.py --config frames --op verify --no-cpu > $O/bench_frames_verify.log 2>&1
timeout -k 10 300 python3 bench.py --config frames --op encode --no-cpu > $O/bench_frames_encode.log 2>&1
echo done
