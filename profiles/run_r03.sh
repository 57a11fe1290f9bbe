#!/bin/bash
# Round-3 GPU pass at HEAD (GPU box, repo root; optional arg: output dir under gpurun_out): GPU tests, the
# bench lines of every config, rocprof kernel stats and PMC HBM traffic per config. Each GPU step has its
# own time limit; the chain stops at the first failure (set -e). The summaries judged are copied to
# profiles/r03 from gpurun_out/<dir>.
set -e
D=${1:-r03}
O=$GRAFT_REPO_ROOT/gpurun_out/$D
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python bench.py --e2e > $O/bench_config1.log 2>&1
timeout -k 10 200 python bench.py --config 2 --steps 20 --warmup 3 --no-cpu > $O/bench_config2.log 2>&1
timeout -k 10 200 python bench.py --config 3 --steps 100 --warmup 10 --e2e > $O/bench_config3_arena.log 2>&1
timeout -k 10 200 python bench.py --config 3 --var-path auto --steps 100 --warmup 10 --no-cpu > $O/bench_config3_auto.log 2>&1
timeout -k 10 200 python bench.py --config 3 --var-path sorted --steps 50 --warmup 5 --no-cpu > $O/bench_config3_sorted.log 2>&1
timeout -k 10 200 python bench.py --config 4 --steps 20 --warmup 3 --no-cpu > $O/bench_config4_n1.log 2>&1
timeout -k 10 200 python bench.py --dist > $O/bench_dist1.log 2>&1
timeout -k 10 200 python bench.py --dist --strong > $O/bench_dist1_strong.log 2>&1
cd /tmp && export TMPDIR=/tmp
for c in 1 2 3; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c$c -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 50 --warmup 5 --no-cpu > $O/kt_c$c.log 2>&1
done
cd $GRAFT_REPO_ROOT
for c in 1 2 3; do
  profiles/pmc.sh $D-c$c --config $c > $O/pmc_c$c.log 2>&1
  python3 profiles/pmc.py gpurun_out/pmc_$D-c$c $O/config${c}_pmc.json > /dev/null
done
echo "r03 pass done"
