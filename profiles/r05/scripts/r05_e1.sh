# Fused encode with coalesced loads and unaligned 16-byte stores: lhc tests + fuzz, then the encode lines.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-e1}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_lhc.py tests/test_gpu_fuzz.py -m gpu > $O/pytest.log 2>&1
for f in mixed chat; do
  timeout -k 10 300 python3 bench.py --config frames --frames $f --op encode --no-cpu > $O/bench_${f}_encode.log 2>&1
done
echo done
