# Sorted path: decode skip + virtual halves zeroed by selects, masks only on edge lines, A/B against the previous commit's library (ANNETY_CRC_LIB), and
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s19}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
BASE=$GRAFT_REPO_ROOT/microbench/base/libannety_crc_0f20181.so
for rep in 1 2 3; do
  PROBES=s timeout -k 10 120 python microbench/stream_probe.py > $O/new_$rep.log 2>&1
  echo "new: $(tail -1 $O/new_$rep.log)" >> $O/ab.log
  ANNETY_CRC_LIB=$BASE PROBES=s timeout -k 10 120 python microbench/stream_probe.py > $O/base_$rep.log 2>&1
  echo "base: $(tail -1 $O/base_$rep.log)" >> $O/ab.log
done
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py::test_config3_full_bitexact tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_var_auto.py tests/test_gpu_arena.py > $O/pytest.log 2>&1
echo done
