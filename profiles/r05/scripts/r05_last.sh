# Last pass at HEAD: every GPU test, smoke(), the default bench line (driver's command) under the tracer and plain,
# the config-3 sorted line.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-last}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1
timeout -k 10 300 python3 bench.py --config 3 --var-path sorted --no-cpu > $O/c3s.log 2>&1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${1:-last}/kt_driver -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/${1:-last}/kt_driver.log 2>&1
echo done
