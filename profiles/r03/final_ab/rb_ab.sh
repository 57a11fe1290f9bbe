#!/bin/bash
# Config 2 (G = 32 nontemporal kernel) at HEAD against 6a3ec9c (before the round-advance byte tables), the
# baseline built in a git worktree; one box, libraries swapped in turn.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-rb}
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for v in rbprev rbhead; do
    cp annety_amd/libannety_crc_$v.so annety_amd/libannety_crc.so
    timeout -k 10 150 python bench.py --config 2 --steps 20 --warmup 3 --no-cpu > $O/c2_${v}_$r.log 2>&1
  done
done
cp annety_amd/libannety_crc_rbhead.so annety_amd/libannety_crc.so
for f in $O/c2_*.log; do echo -n "$f "; tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['frac'])"; done
