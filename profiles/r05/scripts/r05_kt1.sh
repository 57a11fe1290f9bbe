# Kernel trace of the sorted path on config 3 (product kernel through the A/B library, probe 0).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-kt1}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp SORTED_PROBE_CHILD=1 ANNETY_CRC_LIB=$GRAFT_REPO_ROOT/microbench/libannety_crc_ab.so ANNETY_CRC_W8_PROBE=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 microbench/sorted_probe.py > $O/kt.log 2>&1
echo done
