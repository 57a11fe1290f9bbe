# Refresh the lines changed since the final pass: config 3 sorted, frames encode (mixed, chat), PMC of encode.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-refresh}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() { tag=$1; shift; bash profiles/pmc.sh $tag "$@" > $O/pmc_$tag.log 2>&1; python3 profiles/pmc.py gpurun_out/pmc_$tag gpurun_out/pmc_$tag/$tag.json > /dev/null; find gpurun_out/pmc_$tag -name "*counter_collection.csv" -delete; }
run fme --config frames --frames mixed --op encode
run fce --config frames --frames chat --op encode
run c3s --config 3 --var-path sorted
cp gpurun_out/pmc_fme/fme.json gpurun_out/pmc_fce/fce.json gpurun_out/pmc_c3s/c3s.json profiles/r05/pmc/
timeout -k 10 300 python3 bench.py --no-cpu > $O/c1.log 2>&1
timeout -k 10 300 python3 bench.py --config 3 --var-path sorted --no-cpu > $O/c3s.log 2>&1
for f in mixed chat; do timeout -k 10 300 python3 bench.py --config frames --frames $f --op encode --no-cpu > $O/f_${f}_encode.log 2>&1; done
echo done
