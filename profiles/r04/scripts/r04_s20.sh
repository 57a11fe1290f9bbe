# Sorted path, config 3: class order mixing (ANNETY_CRC_SORTED_CLASSES=23: odd blocks run small -> G16 -> G32)
# against the product order (7), and the marginal cost of each class in the fused launch (3 = no small class,
# 5 = no G = 16 class; digests of the skipped class unwritten), alternating.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s20}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for c in 7 23 3 5; do
    ANNETY_CRC_SORTED_CLASSES=$c PROBES=s timeout -k 10 120 python microbench/stream_probe.py > $O/c${c}_$rep.log 2>&1
    echo "classes=$c: $(tail -1 $O/c${c}_$rep.log)" >> $O/ab.log
  done
done
echo done
