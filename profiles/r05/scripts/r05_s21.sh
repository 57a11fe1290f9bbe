# Segment contributions reduced per wave before the atomic: split + sorted tests, then huge / long / config 3 probes.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s21}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sorted_split.py tests/test_gpu_var_layouts.py tests/test_gpu_sorted_edges.py tests/test_gpu_fuzz.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu > $O/pytest.log 2>&1
PROBE_BATCH=huge timeout -k 10 300 python3 microbench/sorted_probe.py 0 > $O/huge.log 2>&1
PROBE_BATCH=long timeout -k 10 300 python3 microbench/sorted_probe.py 0 > $O/long.log 2>&1
timeout -k 10 300 python3 microbench/sorted_probe.py 0 > $O/c3.log 2>&1
echo done
