# Arena stitch with descriptors prefetched one iteration ahead (ANNETY_CRC_STITCH_PIPE=3) against the product
# (PIPE 1), on the config-3 batch and on 2M small frames (BATCH=small), alternating; then the arena parity
# tests under PIPE 3.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s27}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for pp in 1 3; do
    ANNETY_CRC_STITCH_PIPE=$pp PROBES=a timeout -k 10 120 python microbench/stream_probe.py > $O/c3_${pp}_$rep.log 2>&1
    echo "config3 pipe=$pp: $(tail -1 $O/c3_${pp}_$rep.log)" >> $O/ab.log
    ANNETY_CRC_STITCH_PIPE=$pp BATCH=small PROBES=a timeout -k 10 120 python microbench/stream_probe.py > $O/sm_${pp}_$rep.log 2>&1
    echo "small pipe=$pp: $(tail -1 $O/sm_${pp}_$rep.log)" >> $O/ab.log
  done
done
ANNETY_CRC_STITCH_PIPE=3 timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests/test_gpu_arena.py tests/test_gpu_arena_streams.py tests/test_gpu_fullsize.py::test_config3_full_bitexact tests/test_gpu_fuzz.py tests/test_gpu_var_auto.py tests/test_lhc.py > $O/pytest_pipe3.log 2>&1
echo done
