# Sorted path: edge tests at the default, start-aligned rounds A/B (ANNETY_CRC_SORTED_CLASSES bit 32, 55 vs 23)
# with its own parity run, then the default's HBM traffic on config 3 (profiles/pmc.sh passes).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s25}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests/test_gpu_sorted_edges.py > $O/pytest_edges.log 2>&1
for rep in 1 2 3; do
  for c in 23 55; do
    ANNETY_CRC_SORTED_CLASSES=$c PROBES=s timeout -k 10 120 python microbench/stream_probe.py > $O/c${c}_$rep.log 2>&1
    echo "classes=$c: $(tail -1 $O/c${c}_$rep.log)" >> $O/ab.log
  done
done
ANNETY_CRC_SORTED_CLASSES=55 timeout -k 10 300 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests/test_gpu_sorted_edges.py tests/test_gpu_fullsize.py::test_config3_full_bitexact tests/test_gpu_fuzz.py > $O/pytest_sa.log 2>&1
bash profiles/pmc.sh c3s --config 3 --var-path sorted
python3 profiles/pmc.py gpurun_out/pmc_c3s gpurun_out/pmc_c3s/config3_sorted_pmc.json > /dev/null
find gpurun_out/pmc_c3s -name "*counter_collection.csv" -delete
echo done
