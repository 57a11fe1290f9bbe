# Sorted path, config 3: start-aligned rounds in the coalesced classes (ANNETY_CRC_SORTED_CLASSES bit 32)
# against the product (23), alternating; digests checked against the oracle in each run.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s24}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for c in 23 55; do
    ANNETY_CRC_SORTED_CLASSES=$c PROBES=s timeout -k 10 120 python microbench/stream_probe.py > $O/c${c}_$rep.log 2>&1
    echo "classes=$c: $(tail -1 $O/c${c}_$rep.log)" >> $O/ab.log
  done
done
ANNETY_CRC_SORTED_CLASSES=55 timeout -k 10 300 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests/test_gpu_sorted_edges.py tests/test_gpu_fullsize.py::test_config3_full_bitexact tests/test_gpu_fuzz.py > $O/pytest_sa.log 2>&1
echo done
