# Sorted path loader A/B on config 3 (ANNETY_CRC_SORTED_NT bits: 1 = G32 coalesced (default), 3 = G32 + G16),
# alternating; then the full GPU suite at the default, the config-3 sorted bench under the kernel tracer, and
# the driver's default bench command.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s15}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for nt in 1 3; do
    ANNETY_CRC_SORTED_NT=$nt PROBES=s timeout -k 10 120 python microbench/stream_probe.py > $O/ab_${nt}_$rep.log 2>&1
    echo "nt=$nt: $(tail -1 $O/ab_${nt}_$rep.log)" >> $O/ab.log
  done
done
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests > $O/pytest.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c3s -o kt -- python bench.py --config 3 --var-path sorted --steps 50 --warmup 5 > $O/kt_c3s.log 2>&1
timeout -k 10 300 python bench.py --config 3 --var-path sorted > $O/bench_c3s.json 2> $O/bench_c3s.err
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
echo done
