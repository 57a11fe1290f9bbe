# Full GPU suite (the sorted path's G = 32 / 16 classes and the small class at G = 8 now coalesced), then
# bench config 3 --var-path sorted A/B (ANNETY_CRC_SORTED_NT=1 product vs 0 per-line loads), a kernel trace.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s13}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests > $O/pytest.log 2>&1
B="python bench.py --config 3 --var-path sorted --steps 100 --warmup 10 --no-cpu"
for rep in 1 2; do
  ANNETY_CRC_SORTED_NT=1 timeout -k 10 180 $B > $O/nt1_$rep.json 2> $O/nt1_$rep.err
  ANNETY_CRC_SORTED_NT=0 timeout -k 10 180 $B > $O/nt0_$rep.json 2> $O/nt0_$rep.err
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python bench.py --config 3 --var-path sorted --steps 50 --warmup 5 --no-cpu > $O/kt.log 2>&1
echo done
