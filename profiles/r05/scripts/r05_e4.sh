# Encode with three buffers (two steps of loads in flight): lhc tests + fuzz, probes, bench lines.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-e4}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_lhc.py tests/test_gpu_fuzz.py -m gpu > $O/pytest.log 2>&1
timeout -k 10 400 python3 microbench/encode_probe.py 0 1 2 3 > $O/encode_probe.log 2>&1
ENC_FRAMES=chat timeout -k 10 400 python3 microbench/encode_probe.py 0 > $O/encode_probe_chat.log 2>&1
echo done
