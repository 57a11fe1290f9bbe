# Frames verify at three batch sizes: does the stitch's window re-read get cheaper when the stream fits the 256 MB
# Infinity Cache? (kernel-trace per size)
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/mall; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for n in 2097152 262144 131072; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$n -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config frames --frames mixed --op verify --frames-n $n --no-cpu --steps 100 --warmup 10 > $O/b_$n.log 2>&1
done
echo done
