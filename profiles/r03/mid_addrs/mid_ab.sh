#!/bin/bash
# mid-superblock SB addresses stepped from one division (this build) against one division each (libannety_crc_prev.so, the previous
# commit): arena/frame GPU tests, then config-3 bench lines alternating on one box by swapping the library.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-mid}
mkdir -p $O
cd $GRAFT_REPO_ROOT
cp annety_amd/libannety_crc.so annety_amd/libannety_crc_new.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_arena.py tests/test_gpu_nt.py tests/test_gpu_var_auto.py tests/test_gpu_arena_streams.py tests/test_lhc.py tests/test_gpu_fuzz.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
for r in 1 2 3; do
  cp annety_amd/libannety_crc_new.so annety_amd/libannety_crc.so
  timeout -k 10 150 python bench.py --config 3 --steps 200 --warmup 20 --no-cpu > $O/c3_new_$r.log 2>&1
  cp annety_amd/libannety_crc_prev.so annety_amd/libannety_crc.so
  timeout -k 10 150 python bench.py --config 3 --steps 200 --warmup 20 --no-cpu > $O/c3_prev_$r.log 2>&1
done
cp annety_amd/libannety_crc_new.so annety_amd/libannety_crc.so
for f in $O/c3_*.log; do echo -n "$f "; tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['frac'])"; done
