# Sorted path, config 3: small class with two steps of loads in flight (bit 32) and class-order mixing (bit 16),
# against the product (7), alternating.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s21}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for c in 7 23 39 55; do
    ANNETY_CRC_SORTED_CLASSES=$c PROBES=s timeout -k 10 120 python microbench/stream_probe.py > $O/c${c}_$rep.log 2>&1
    echo "classes=$c: $(tail -1 $O/c${c}_$rep.log)" >> $O/ab.log
  done
done
echo done
