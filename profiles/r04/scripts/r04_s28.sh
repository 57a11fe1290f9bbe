# Sorted path, config 3: the >= 128-line class at G = 16 (ANNETY_CRC_SORTED_CLASSES bit 64: 87) against G = 32
# (23), alternating, digests checked.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s28}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for c in 23 87; do
    ANNETY_CRC_SORTED_CLASSES=$c PROBES=s timeout -k 10 120 python microbench/stream_probe.py > $O/c${c}_$rep.log 2>&1
    echo "classes=$c: $(tail -1 $O/c${c}_$rep.log)" >> $O/ab.log
  done
done
echo done
