# Last pass of round 4: the full GPU suite and smoke at HEAD, then the sorted path (23) on config 3.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s29}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
for rep in 1 2 3; do
  for c in 23; do
    ANNETY_CRC_SORTED_CLASSES=$c PROBES=s timeout -k 10 120 python microbench/stream_probe.py > $O/c${c}_$rep.log 2>&1
    echo "classes=$c: $(tail -1 $O/c${c}_$rep.log)" >> $O/ab.log
  done
done
echo done
