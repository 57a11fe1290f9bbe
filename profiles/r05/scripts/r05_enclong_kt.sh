# Kernel times of the long-frame encode (16 x 64 MiB; 256 x 1 MiB among 200K short).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/enclong_kt; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for kind in long longmix; do
  ENC_FRAMES=$kind ENC_CALLS=5 ENC_PROBE_CHILD=1 ANNETY_CRC_LIB=$GRAFT_REPO_ROOT/microbench/libannety_crc_ab.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$kind -o run -- python3 $GRAFT_REPO_ROOT/microbench/encode_probe.py > $O/$kind.log 2>&1
done
echo done
