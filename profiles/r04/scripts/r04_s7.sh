set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s7}; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -v --timeout 200 --timeout-method thread > $O/pytest_stream.log 2>&1
timeout -k 10 300 python microbench/stream_probe.py > $O/probe.log 2>&1
timeout -k 10 150 python bench.py --config 3 --var-path stream --steps 100 --warmup 10 --no-cpu > $O/bench_stream.log 2>&1
echo done
