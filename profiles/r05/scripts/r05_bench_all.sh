# Every bench line at HEAD (one box): configs 1-4, config 3 on the sorted path, the four frames lines.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-bench}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --no-cpu > $O/c1.log 2>&1
timeout -k 10 300 python3 bench.py --config 2 --no-cpu > $O/c2.log 2>&1
timeout -k 10 300 python3 bench.py --config 3 --no-cpu > $O/c3.log 2>&1
timeout -k 10 300 python3 bench.py --config 3 --var-path sorted --no-cpu > $O/c3s.log 2>&1
timeout -k 10 300 python3 bench.py --config 4 --no-cpu > $O/c4.log 2>&1
for f in mixed chat; do for op in verify encode; do
  timeout -k 10 300 python3 bench.py --config frames --frames $f --op $op --no-cpu > $O/f_${f}_${op}.log 2>&1
done; done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c3s -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config 3 --var-path sorted --no-cpu > $O/kt_c3s.log 2>&1
echo done
