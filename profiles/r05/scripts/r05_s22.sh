# Same-box A/B, config 3 sorted: the wave-reduced segment atomics (new) against the per-group atomics (prev).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s22}; mkdir -p $O; cd $GRAFT_REPO_ROOT
for rep in 0 1 2; do
  PROBE_LIB=$GRAFT_REPO_ROOT/microbench/libannety_crc_ab_prev.so timeout -k 10 200 python3 microbench/sorted_probe.py 0 > $O/prev_$rep.log 2>&1
  PROBE_LIB=$GRAFT_REPO_ROOT/microbench/libannety_crc_ab.so timeout -k 10 200 python3 microbench/sorted_probe.py 0 > $O/new_$rep.log 2>&1
done
echo done
