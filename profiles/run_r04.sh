#!/bin/bash
# Round-4 GPU pass (GPU box, repo root; arg 1: output dir under gpurun_out, arg 2: "tests" to run the GPU
# suite and smoke first). Then the driver's exact bench command, its rocprofv3 kernel trace (same command, so
# the committed average and the line's frac come from one box), PMC HBM traffic per config, and the other
# configs' lines. Each GPU step has its own time limit; the chain stops at the first failure (set -e).
set -e
D=${1:-r04}
O=$GRAFT_REPO_ROOT/gpurun_out/$D
mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ "$2" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
fi
# the driver's command, then the same command under the kernel trace
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_driver -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $O/kt_driver.log 2>&1
cd $GRAFT_REPO_ROOT
for c in 2 3; do
  timeout -k 10 200 python bench.py --config $c --steps 50 --warmup 5 --no-cpu > $O/bench_config$c.log 2>&1
done
timeout -k 10 200 python bench.py --config 3 --var-path sorted --steps 50 --warmup 5 --no-cpu > $O/bench_config3_sorted.log 2>&1
cd /tmp
for c in 2 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c$c -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 50 --warmup 5 --no-cpu > $O/kt_c$c.log 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c3sorted -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --config 3 --var-path sorted --steps 50 --warmup 5 --no-cpu > $O/kt_c3sorted.log 2>&1
cd $GRAFT_REPO_ROOT
for c in 1 2 3; do
  profiles/pmc.sh $D-c$c --config $c > $O/pmc_c$c.log 2>&1
  python3 profiles/pmc.py gpurun_out/pmc_$D-c$c $O/config${c}_pmc.json > /dev/null
done
echo "r04 pass done"
