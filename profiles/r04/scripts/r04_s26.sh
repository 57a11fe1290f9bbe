# Small frames (2M payloads of 16 B - 1 KiB, packed, shuffled: BATCH=small) and the config-3 batch: automatic
# choice (u) against the sorted (s) and arena (a) entries, alternating; digests checked in every run.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s26}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
BATCH=small PROBES="u s a u s a" timeout -k 10 300 python microbench/stream_probe.py > $O/small.log 2>&1
PROBES="u s a u s a" timeout -k 10 300 python microbench/stream_probe.py > $O/config3.log 2>&1
echo done
