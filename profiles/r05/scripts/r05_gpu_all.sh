# Round-5 GPU pass at HEAD: every GPU test, smoke(), the default bench line and its kernel trace.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-all}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 300 python3 bench.py > $O/bench_default.log 2>&1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_default -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu > $O/kt_default.log 2>&1
echo done
