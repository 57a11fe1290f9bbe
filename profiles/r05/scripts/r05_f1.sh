# Frames regime lines (bench --config frames): verify and encode, mixed (16 B-1 KiB) and chat (408 B), then a
# kernel trace of each.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-f1}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_lhc.py -m gpu > $O/pytest_lhc.log 2>&1
for f in mixed chat; do for op in verify encode; do
  timeout -k 10 300 python3 bench.py --config frames --frames $f --op $op --no-cpu > $O/bench_${f}_${op}.log 2>&1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${f}_${op} -o run -- python3 bench.py --config frames --frames $f --op $op --no-cpu --steps 20 --warmup 5 > $O/kt_${f}_${op}.log 2>&1
done; done
echo done
