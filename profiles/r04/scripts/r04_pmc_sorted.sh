# HBM traffic of the sorted path on config 3 at HEAD (profiles/pmc.sh passes, summarised on the box).
set -e
cd $GRAFT_REPO_ROOT
bash profiles/pmc.sh c3s --config 3 --var-path sorted
python3 profiles/pmc.py gpurun_out/pmc_c3s gpurun_out/pmc_c3s/config3_sorted_pmc.json
find gpurun_out/pmc_c3s -name "*counter_collection.csv" -delete
echo done
