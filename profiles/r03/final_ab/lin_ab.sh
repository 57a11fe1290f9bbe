#!/bin/bash
# Linear SB with stepped mid-superblock indices (lin, this build) against cb30984, one box, libraries swapped.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-lin}
mkdir -p $O
cd $GRAFT_REPO_ROOT
cp annety_amd/libannety_crc_lin.so annety_amd/libannety_crc.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_arena.py tests/test_gpu_nt.py tests/test_gpu_var_auto.py tests/test_gpu_arena_streams.py tests/test_lhc.py tests/test_gpu_fuzz.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
for r in 1 2 3; do
  for v in cb30984 lin; do
    cp annety_amd/libannety_crc_$v.so annety_amd/libannety_crc.so
    timeout -k 10 150 python bench.py --config 3 --steps 200 --warmup 20 --no-cpu > $O/c3_${v}_$r.log 2>&1
  done
done
cp annety_amd/libannety_crc_lin.so annety_amd/libannety_crc.so
tail -1 $O/pytest.log
for f in $O/c3_*.log; do echo -n "$f "; tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['frac'])"; done
