# Full GPU suite, then the stitch's superblock join A/B (chain + PIPE 1 = product, one level = MID 1, chain
# without PIPE) on config 3 and on long payloads, under the kernel tracer.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s11}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
for b in zipf long; do
  for m in prod mid nopipe prod mid; do
    unset ANNETY_CRC_STITCH_MID ANNETY_CRC_STITCH_PIPE
    [ $m = mid ] && export ANNETY_CRC_STITCH_MID=1
    [ $m = nopipe ] && export ANNETY_CRC_STITCH_PIPE=0
    BATCH=$b PROBES=a timeout -k 10 120 python microbench/stream_probe.py >> $O/stitch_ab_$b.log 2>&1
    echo "$b $m: $(tail -1 $O/stitch_ab_$b.log)" >> $O/stitch_ab.log
  done
done
unset ANNETY_CRC_STITCH_MID ANNETY_CRC_STITCH_PIPE
for m in prod mid; do
  [ $m = mid ] && export ANNETY_CRC_STITCH_MID=1
  PROBES=a timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/kt_$m -o kt -- python microbench/stream_probe.py > $O/kt_$m.log 2>&1
done
echo done
