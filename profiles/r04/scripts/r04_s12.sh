# Full GPU suite (the sorted path's G = 32 / 16 classes now coalesced), then
# bench config 3 --var-path sorted A/B (ANNETY_CRC_SORTED_NT=1 product vs 0 per-line loads), a kernel trace,
# and the stitch's superblock join A/B (chain = product, one level = ANNETY_CRC_STITCH_MID=1).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s12}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests > $O/pytest.log 2>&1
B="python bench.py --config 3 --var-path sorted --steps 100 --warmup 10 --no-cpu"
for rep in 1 2; do
  ANNETY_CRC_SORTED_NT=1 timeout -k 10 180 $B > $O/nt1_$rep.json 2> $O/nt1_$rep.err
  ANNETY_CRC_SORTED_NT=0 timeout -k 10 180 $B > $O/nt0_$rep.json 2> $O/nt0_$rep.err
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python bench.py --config 3 --var-path sorted --steps 50 --warmup 5 --no-cpu > $O/kt.log 2>&1
for b in zipf long; do
  for m in prod mid prod mid; do
    unset ANNETY_CRC_STITCH_MID
    [ $m = mid ] && export ANNETY_CRC_STITCH_MID=1
    BATCH=$b PROBES=a timeout -k 10 120 python microbench/stream_probe.py >> $O/stitch_ab_$b.log 2>&1
    echo "$b $m: $(tail -1 $O/stitch_ab_$b.log)" >> $O/stitch_ab.log
  done
done
echo done
