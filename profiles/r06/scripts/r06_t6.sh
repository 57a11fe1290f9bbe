# Auto-path tests + the fresh/stable/sorted probe after the record fix and the extent kernel change.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-t6}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_var_auto.py tests/test_gpu_sorted_split.py tests/test_gpu_arena.py -x -v -s --timeout 200 --timeout-method thread > $O/auto.log 2>&1
timeout -k 10 300 python3 -u microbench/auto_fresh_probe.py 20 > $O/probe.log 2>&1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
   python3 $GRAFT_REPO_ROOT/microbench/auto_fresh_probe.py 12 > $O/probe_kt.log 2>&1)
find $O/kt -name "*kernel_trace.csv" -size +2M -delete
echo done
