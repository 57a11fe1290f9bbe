# Long-frame encode after the per-segment copy: tests, then per-call time (new build only), then the encode bench lines.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/enclong3; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_encode_long.py tests/test_lhc.py -m gpu > $O/pytest.log 2>&1
for kind in long longmix; do
  echo "== $kind" >> $O/probe.log
  ENC_FRAMES=$kind ENC_CALLS=20 timeout -k 10 250 python3 microbench/encode_probe.py 0 >> $O/probe.log 2>&1
done
timeout -k 10 200 python3 bench.py --config frames --frames chat --op encode --no-cpu > $O/b_chat.log 2>&1
echo done
