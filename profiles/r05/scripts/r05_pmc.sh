# HBM traffic (profiles/pmc.sh passes, summarised on the box) of the kernels that changed in round 5.
set -e
cd $GRAFT_REPO_ROOT
run() { tag=$1; shift; bash profiles/pmc.sh $tag "$@"; python3 profiles/pmc.py gpurun_out/pmc_$tag gpurun_out/pmc_$tag/$tag.json > /dev/null; find gpurun_out/pmc_$tag -name "*counter_collection.csv" -delete; }
run c3s --config 3 --var-path sorted
run c3a --config 3
run fmv --config frames --frames mixed --op verify
run fme --config frames --frames mixed --op encode
run fcv --config frames --frames chat --op verify
run fce --config frames --frames chat --op encode
echo done
