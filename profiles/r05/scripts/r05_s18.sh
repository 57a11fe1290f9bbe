# Long payloads split into segments on the sorted path: new split tests + the sorted/fuzz/fullsize suites, then the
# long-payload probe and config 3.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s18}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sorted_split.py tests/test_gpu_var_layouts.py tests/test_gpu_sorted_edges.py tests/test_gpu_fuzz.py tests/test_gpu_fullsize.py tests/test_gpu_var_auto.py tests/test_gpu_parity.py -m gpu > $O/pytest.log 2>&1
PROBE_BATCH=long timeout -k 10 300 python3 microbench/sorted_probe.py 0 > $O/long.log 2>&1
timeout -k 10 300 python3 microbench/sorted_probe.py 0 > $O/c3.log 2>&1
echo done
