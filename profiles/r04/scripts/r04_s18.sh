# Sorted path: descriptor decode skipped while every group continues its task, A/B against the previous commit's library (ANNETY_CRC_LIB), and
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s18}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
BASE=$GRAFT_REPO_ROOT/microbench/base/libannety_crc_0f20181.so
for rep in 1 2 3; do
  PROBES=s timeout -k 10 120 python microbench/stream_probe.py > $O/new_$rep.log 2>&1
  echo "new: $(tail -1 $O/new_$rep.log)" >> $O/ab.log
  ANNETY_CRC_LIB=$BASE PROBES=s timeout -k 10 120 python microbench/stream_probe.py > $O/base_$rep.log 2>&1
  echo "base: $(tail -1 $O/base_$rep.log)" >> $O/ab.log
done
echo done
