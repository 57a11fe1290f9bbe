# Round-5 final pass at HEAD: every GPU test, smoke(), PMC traffic of the kernels changed since the last pass,
# every bench line, kernel traces of the default and the sorted-path lines.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-final}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
run() { tag=$1; shift; bash profiles/pmc.sh $tag "$@" > $O/pmc_$tag.log 2>&1; python3 profiles/pmc.py gpurun_out/pmc_$tag gpurun_out/pmc_$tag/$tag.json > /dev/null; find gpurun_out/pmc_$tag -name "*counter_collection.csv" -delete; }
run c3s --config 3 --var-path sorted
run fme --config frames --frames mixed --op encode
run fce --config frames --frames chat --op encode
cp gpurun_out/pmc_c3s/c3s.json gpurun_out/pmc_fme/fme.json gpurun_out/pmc_fce/fce.json profiles/r05/pmc/
timeout -k 10 300 python3 bench.py > $O/bench_default.log 2>&1
bash profiles/r05/scripts/r05_bench_all.sh ${1:-final}/bench
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_default -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu > $O/kt_default.log 2>&1
echo done
