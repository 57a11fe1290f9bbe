# Table-driven chunk masks (mask_chunks): sorted + lhc + fuzz + fullsize tests, then sorted/encode probes.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s14}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_var_layouts.py tests/test_gpu_sorted_edges.py tests/test_gpu_fuzz.py tests/test_gpu_fullsize.py tests/test_lhc.py tests/test_gpu_var_auto.py -m gpu > $O/pytest.log 2>&1
timeout -k 10 300 python3 microbench/sorted_probe.py 0 16 > $O/c3.log 2>&1
PROBE_BATCH=small timeout -k 10 300 python3 microbench/sorted_probe.py 0 16 > $O/small.log 2>&1
timeout -k 10 300 python3 microbench/encode_probe.py 0 1 > $O/encode.log 2>&1
echo done
