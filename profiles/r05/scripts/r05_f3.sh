# Stitch windows: only the 16-byte chunks with kept bytes read the batch. Tests, frames verify lines, config 3 arena.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-f3}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_lhc.py tests/test_gpu_fuzz.py tests/test_gpu_arena.py tests/test_gpu_parity.py -m gpu > $O/pytest.log 2>&1
for f in mixed chat; do
  timeout -k 10 300 python3 bench.py --config frames --frames $f --op verify --no-cpu > $O/bench_${f}_verify.log 2>&1
done
timeout -k 10 300 python3 bench.py --config 3 --no-cpu > $O/bench_c3_auto.log 2>&1
echo done
