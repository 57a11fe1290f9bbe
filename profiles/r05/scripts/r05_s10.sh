# 2M packed payloads of 16 B - 1 KiB (the frames regime's payloads): sorted path against the arena (auto).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s10}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PROBE_BATCH=small
PROBE_PATH=sorted timeout -k 10 300 python3 microbench/sorted_probe.py 0 1 2 > $O/small_sorted.log 2>&1
PROBE_PATH=auto timeout -k 10 300 python3 microbench/sorted_probe.py 0 > $O/small_auto.log 2>&1
echo done
