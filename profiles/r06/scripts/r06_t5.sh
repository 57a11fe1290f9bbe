# The whole GPU suite, timing prints of the new tests, the default bench line.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-t5}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -u -m pytest -s -q --timeout 200 --timeout-method thread \
  tests/test_gpu_sorted_split.py::test_update_mode_split_16x64mib tests/test_gpu_var_auto.py::test_fresh_pointers_reach_the_arena \
  tests/test_gpu_arena_long.py::test_verify_stream_64mib_frames > $O/timing_tests.log 2>&1
timeout -k 10 300 python3 bench.py > $O/bench_default.log 2>&1
echo done
