# The driver's exact default command on one box: plain, then under rocprofv3 --kernel-trace --stats (the headline's
# kernel average from the profiler beside the bench line's own HIP-event figure).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-defkt}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py > $O/bench_default.log 2>&1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_default -o run -- python3 $GRAFT_REPO_ROOT/bench.py > $O/bench_default_under_rocprof.log 2>&1)
find $O/kt_default -name "*kernel_trace.csv" -delete
python3 profiles/r06/kt_summary.py $O/kt_default $O/kt_default.csv
grep -o '"frac": [0-9.]*\|"kernel_ms_avg": [0-9.]*\|"value": [0-9.]*' $O/bench_default.log $O/bench_default_under_rocprof.log
