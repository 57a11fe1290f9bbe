# A/B: stitch waves of short payloads skip the block-run and mid loads (ANNETY_CRC_STITCH_PROBE=6, correct digests)
# against the product, frames verify (mixed, chat; the bench checks every verdict first) and config 3, twice.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-abshort}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp ANNETY_CRC_LIB=$GRAFT_REPO_ROOT/microbench/libannety_crc_ab.so
for rep in 1 2; do
  for pr in 0 6; do
    for line in "--config frames --frames mixed --op verify" "--config frames --frames chat --op verify" "--config 3 --var-path arena"; do
      tag=$(echo "$line" | tr -d ' -' | cut -c1-24)
      ANNETY_CRC_STITCH_PROBE=$pr timeout -k 10 200 python3 bench.py $line --steps 200 --warmup 20 --no-cpu > $O/r${rep}_p${pr}_$tag.log 2>&1
      echo "rep $rep probe $pr $tag $(grep -o '"ms_per_step": [0-9.]*' $O/r${rep}_p${pr}_$tag.log)"
    done
  done
done
