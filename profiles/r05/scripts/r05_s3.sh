# var_class_w8 with the descriptor fetched a whole task ahead: sorted-path parity, then stage probes.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s3}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_var_layouts.py tests/test_gpu_sorted_edges.py > $O/pytest_sorted.log 2>&1
timeout -k 10 500 python3 microbench/sorted_probe.py 3:0 1:0 2:0 3:1 3:2 > $O/sorted_probe.log 2>&1
echo done
