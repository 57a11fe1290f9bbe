# What the byte masks cost in the sorted path's masked rounds (W8 probe 16), config 3 and 2M small payloads.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s13}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 microbench/sorted_probe.py 0 16 1 > $O/c3.log 2>&1
PROBE_BATCH=small timeout -k 10 300 python3 microbench/sorted_probe.py 0 16 1 > $O/small.log 2>&1
echo done
