#!/bin/bash
# Config 4 under sustained load with the GPU's clocks, power and temperatures sampled every second
# (rocm-smi, read-only), to tell a power limit from a thermal one. GPU box, repo root.
O=$GRAFT_REPO_ROOT/gpurun_out/c4watch
mkdir -p $O
( for i in $(seq 1 150); do date +%s.%N; rocm-smi --showpower --showtemp --showclocks --showuse 2>/dev/null; sleep 1; done ) > $O/smi.log 2>&1 &
W=$!
timeout -k 10 60 python bench.py --config 4 --steps 20 --warmup 3 --no-cpu > $O/c4_first.log 2>&1
timeout -k 10 120 python bench.py --config 4 --steps 2000 --warmup 3 --no-cpu --prewarm-s 0 > $O/c4_long.log 2>&1
timeout -k 10 60 python bench.py --config 4 --steps 20 --warmup 3 --no-cpu > $O/c4_after.log 2>&1
rc=$?
kill $W 2>/dev/null
exit $rc
