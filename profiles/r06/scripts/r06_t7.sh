# The whole GPU suite + smoke, then the lines whose kernels changed since the checkpoint (arena unit).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-t7}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
bash profiles/r06/scripts/r06_measure.sh ${1:-t7}/m c3a c3s fmv fcv
echo done
