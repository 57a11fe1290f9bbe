#!/bin/bash
# Round-2 GPU pass (run on the box from the repo root; optional arg: output dir under gpurun_out): tests, bench lines for every config, rocprof
# kernel stats and PMC traffic at this code. Each GPU step has its own time limit; the chain stops at
# the first failure (set -e). Outputs under gpurun_out/r02; the summaries judged are copied to profiles/r02.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r02}
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --e2e > $O/bench_config1.log 2>&1
timeout -k 10 200 python bench.py --config 2 --steps 20 --warmup 3 --no-cpu > $O/bench_config2.log 2>&1
timeout -k 10 200 python bench.py --config 3 --steps 50 --warmup 5 --e2e > $O/bench_config3_arena.log 2>&1
timeout -k 10 200 python bench.py --config 3 --var-path sorted --steps 50 --warmup 5 --no-cpu > $O/bench_config3_sorted.log 2>&1
timeout -k 10 200 python bench.py --config 4 --steps 20 --warmup 3 --no-cpu > $O/bench_config4_n1.log 2>&1
timeout -k 10 200 python bench.py --dist --steps 100 --warmup 5 > $O/bench_config4_dist1.log 2>&1
cd /tmp && export TMPDIR=/tmp
for c in 1 2 3; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c$c -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 50 --warmup 5 --no-cpu > $O/kt_c$c.log 2>&1
done
cd $GRAFT_REPO_ROOT
for c in 1 2 3; do
  profiles/pmc.sh c$c --config $c > $O/pmc_c$c.log 2>&1
  python3 profiles/pmc.py gpurun_out/pmc_c$c $O/config${c}_pmc.json > /dev/null
done
echo "r02 pass done"
