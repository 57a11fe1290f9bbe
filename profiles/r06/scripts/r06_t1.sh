# GPU suite at HEAD (update-mode split, split cap) + the default bench line.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-t1}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python3 bench.py > $O/bench_default.log 2>&1
echo done
