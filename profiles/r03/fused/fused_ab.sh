set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fz
timeout -k 10 400 python -u -m pytest tests/test_gpu_arena.py tests/test_gpu_nt.py tests/test_gpu_var_auto.py tests/test_gpu_arena_streams.py tests/test_lhc.py tests/test_gpu_fuzz.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/fz/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/fz/pytest.log; exit 1; }
tail -2 gpurun_out/fz/pytest.log
for i in 1 2; do
  timeout -k 10 150 python bench.py --config 3 --steps 200 --warmup 20 --no-cpu > gpurun_out/fz/c3_fused_$i.log 2>&1 || exit 2
  ANNETY_CRC_ARENA_FUSED=0 timeout -k 10 150 python bench.py --config 3 --steps 200 --warmup 20 --no-cpu > gpurun_out/fz/c3_two_$i.log 2>&1 || exit 3
done
for f in gpurun_out/fz/c3_*.log; do echo $f; tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['frac'])"; done
