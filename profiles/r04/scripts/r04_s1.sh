set -e
O=$GRAFT_REPO_ROOT/gpurun_out/s1; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py -x -v --timeout 200 --timeout-method thread > $O/pytest_stream.log 2>&1
for p in stream sorted arena; do
  timeout -k 10 150 python bench.py --config 3 --var-path $p --steps 100 --warmup 10 --no-cpu > $O/bench_$p.log 2>&1
done
echo done
