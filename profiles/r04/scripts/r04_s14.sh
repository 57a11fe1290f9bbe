# Sorted path per-class times (ANNETY_CRC_SORTED_CLASSES: one class alone; digests of the others unwritten) for
# the three loader variants (ANNETY_CRC_SORTED_NT 1 = product, 0 = per-line, 2 = small class at G = 8), then
# the scale-prediction inputs (profiles/r04/scripts/r04_scale_inputs.sh).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s14}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for nt in 1 0 2; do
  for c in 7 1 2 4; do
    ANNETY_CRC_SORTED_NT=$nt ANNETY_CRC_SORTED_CLASSES=$c PROBES=s timeout -k 10 120 python microbench/stream_probe.py > $O/cls_${nt}_$c.log 2>&1
    echo "nt=$nt classes=$c: $(tail -1 $O/cls_${nt}_$c.log)" >> $O/classes.log
  done
done
bash profiles/r04/scripts/r04_scale_inputs.sh ${1:-s14}/scale
echo done
