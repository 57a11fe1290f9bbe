# What the stitch's S/SB word loads (probe 4) and window loads (probe 5) cost: A/B build, arena path, 2M small
# payloads (PROBE_BATCH=small) and config 3 (default batch); microseconds per call.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-probes}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PROBE_PATH=auto
PROBE_BATCH=small timeout -k 10 400 python3 microbench/sorted_probe.py 0 4 5 > $O/small.log 2>&1
cat $O/small.log
timeout -k 10 400 python3 microbench/sorted_probe.py 0 4 5 > $O/c3.log 2>&1
cat $O/c3.log
