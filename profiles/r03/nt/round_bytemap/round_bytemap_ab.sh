#!/bin/bash
# G = 32 round advance through byte tables (this build) against the nibble map (libannety_crc_prev.so, the
# previous commit), config 2 bench lines alternating on one box by swapping the library file.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-rbm}
mkdir -p $O
cd $GRAFT_REPO_ROOT/annety_amd
cp libannety_crc.so libannety_crc_new.so
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  cp annety_amd/libannety_crc_new.so annety_amd/libannety_crc.so
  timeout -k 10 200 python bench.py --config 2 --steps 20 --warmup 3 --no-cpu > $O/c2_new_$r.log 2>&1
  cp annety_amd/libannety_crc_prev.so annety_amd/libannety_crc.so
  timeout -k 10 200 python bench.py --config 2 --steps 20 --warmup 3 --no-cpu > $O/c2_prev_$r.log 2>&1
done
cp annety_amd/libannety_crc_new.so annety_amd/libannety_crc.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_nt.py tests/test_gpu_fullsize.py -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
echo done
