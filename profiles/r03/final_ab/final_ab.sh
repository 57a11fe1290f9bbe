#!/bin/bash
# Config 3 at HEAD against the two commits before this session's arena changes, one box, libraries swapped
# in turn: cb30984 (before SB bursts), 2971e7c (SB bursts), head (+ stepped mid-superblock indices).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-fab}
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for v in cb30984 2971e7c head; do
    cp annety_amd/libannety_crc_$v.so annety_amd/libannety_crc.so
    timeout -k 10 150 python bench.py --config 3 --steps 200 --warmup 20 --no-cpu > $O/c3_${v}_$r.log 2>&1
  done
done
cp annety_amd/libannety_crc_head.so annety_amd/libannety_crc.so
for f in $O/c3_*.log; do echo -n "$f "; tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['frac'], d['roofline']['achieved'])"; done
