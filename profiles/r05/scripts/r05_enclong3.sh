# Long-frame encode: tests, then kernel times (16 x 64 MiB; 256 x 1 MiB among 200K short), then the chat encode line.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-enclong4}; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_encode_long.py tests/test_lhc.py -m gpu > $O/pytest.log 2>&1
cd /tmp && export TMPDIR=/tmp
for kind in long longmix; do
  ENC_FRAMES=$kind ENC_CALLS=5 ENC_PROBE_CHILD=1 ANNETY_CRC_LIB=$GRAFT_REPO_ROOT/microbench/libannety_crc_ab.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$kind -o run -- python3 $GRAFT_REPO_ROOT/microbench/encode_probe.py > $O/$kind.log 2>&1
done
cd $GRAFT_REPO_ROOT && timeout -k 10 200 python3 bench.py --config frames --frames chat --op encode --no-cpu > $O/b_chat.log 2>&1
echo done
