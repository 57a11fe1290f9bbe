# The automatic path with fresh pointers per call (device choice) vs stable pointers vs the sorted path: event and
# host timings, then the same under a kernel trace.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-fresh}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u microbench/auto_fresh_probe.py 20 > $O/probe.log 2>&1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
   python3 $GRAFT_REPO_ROOT/microbench/auto_fresh_probe.py 12 > $O/probe_kt.log 2>&1)
find $O/kt -name "*kernel_trace.csv" -size +2M -delete
echo done
