# The arena join with partial-wave-safe sharing: the partial-ends loop (progress per call), then the arena tests.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-t3}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u microbench/dbg_partial.py > $O/dbg.log 2>&1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_arena.py tests/test_gpu_arena_long.py -x -v -s --timeout 200 --timeout-method thread > $O/arena.log 2>&1
echo done
