# Frames verify with the trailer compare fused into the stitch: lhc tests, fuzz round trips, bench lines + trace.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-f2}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_lhc.py tests/test_gpu_fuzz.py tests/test_gpu_arena.py -m gpu > $O/pytest_lhc.log 2>&1
for f in mixed chat; do
  timeout -k 10 300 python3 bench.py --config frames --frames $f --op verify --no-cpu > $O/bench_${f}_verify.log 2>&1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${f}_verify -o run -- python3 bench.py --config frames --frames $f --op verify --no-cpu --steps 20 --warmup 5 > $O/kt_${f}_verify.log 2>&1
done
echo done
