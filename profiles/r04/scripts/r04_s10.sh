set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s10}; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 600 python microbench/stream_probe.py > $O/probe.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python bench.py --config 3 > $O/bench_c3.json 2> $O/bench_c3.err
timeout -k 10 300 python bench.py --config 3 --var-path sorted > $O/bench_c3s.json 2> $O/bench_c3s.err
echo done
