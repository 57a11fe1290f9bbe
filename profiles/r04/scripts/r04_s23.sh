# Sorted-path edge tests (tests/test_gpu_sorted_edges.py), then its HBM traffic on config 3 at HEAD
# (profiles/pmc.sh passes, summarised on the box).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s23
timeout -k 10 300 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests/test_gpu_sorted_edges.py > gpurun_out/s23/pytest.log 2>&1
bash profiles/pmc.sh c3s --config 3 --var-path sorted
python3 profiles/pmc.py gpurun_out/pmc_c3s gpurun_out/pmc_c3s/config3_sorted_pmc.json
find gpurun_out/pmc_c3s -name "*counter_collection.csv" -delete
echo done
