# Stitch stage costs on 2M packed payloads of 16 B - 1 KiB (arena path): PROBE 0 (product) 1 2 3.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s11}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PROBE_BATCH=small PROBE_PATH=auto
timeout -k 10 300 python3 microbench/sorted_probe.py 0 1 2 3 > $O/small_stitch_probe.log 2>&1
echo done
