# Sorted path as one list (every payload in var_class_w8, claim ring in LDS): sorted parity, fuzz, then probes.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s6}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_var_layouts.py tests/test_gpu_sorted_edges.py tests/test_gpu_fuzz.py tests/test_gpu_fullsize.py > $O/pytest_sorted.log 2>&1
timeout -k 10 300 python3 microbench/sorted_probe.py 0 1 2 > $O/sorted_probe.log 2>&1
echo done
