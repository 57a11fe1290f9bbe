# Long-frame encode: per-call time before (the previous build) and after the long path.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/enclong_perf; mkdir -p $O; cd $GRAFT_REPO_ROOT
for kind in long longmix; do
  for lib in libannety_crc_ab_prev.so libannety_crc_ab.so; do
    echo "== $kind $lib" >> $O/probe.log
    ENC_FRAMES=$kind ENC_CALLS=$([ $kind = long ] && echo 3 || echo 20) ENC_LIB=$GRAFT_REPO_ROOT/microbench/$lib timeout -k 10 250 python3 microbench/encode_probe.py 0 >> $O/probe.log 2>&1
  done
done
echo done
