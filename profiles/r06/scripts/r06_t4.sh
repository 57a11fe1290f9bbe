# Arena tests with the wave-per-payload stitch for few payloads, then the whole GPU suite, then timing prints.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-t4}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_arena.py tests/test_gpu_arena_long.py -x -v -s --timeout 200 --timeout-method thread > $O/arena.log 2>&1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -u -m pytest -s -q --timeout 200 --timeout-method thread \
  tests/test_gpu_sorted_split.py::test_update_mode_split_16x64mib tests/test_gpu_var_auto.py::test_fresh_pointers_reach_the_arena \
  > $O/timing_tests.log 2>&1
timeout -k 10 300 python3 bench.py > $O/bench_default.log 2>&1
echo done
