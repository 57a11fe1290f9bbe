# Encode long frames: the new tests, the existing encode tests, the frames encode bench lines (kernel trace).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/enclong; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_encode_long.py tests/test_lhc.py tests/test_pbc.py -m gpu > $O/pytest.log 2>&1
timeout -k 10 200 python3 bench.py --config frames --frames mixed --op encode --no-cpu > $O/b_mixed.log 2>&1
timeout -k 10 200 python3 bench.py --config frames --frames chat --op encode --no-cpu > $O/b_chat.log 2>&1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config frames --frames mixed --op encode --no-cpu --steps 50 --warmup 5 > $O/kt.log 2>&1
echo done
