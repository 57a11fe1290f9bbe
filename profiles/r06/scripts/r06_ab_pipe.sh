# A/B of the stitch's payload pipeline (ANNETY_CRC_STITCH_PIPE 1 = product, 3 = descriptors a round ahead, every
# load unconditional) on the A/B build, frames verify (mixed, chat) and config 3 arena, alternating twice.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-abpipe}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp ANNETY_CRC_LIB=$GRAFT_REPO_ROOT/microbench/libannety_crc_ab.so
for rep in 1 2; do
  for pipe in 1 3; do
    for line in "--config frames --frames mixed --op verify" "--config frames --frames chat --op verify" "--config 3 --var-path arena"; do
      tag=$(echo "$line" | tr -d ' -' | cut -c1-24)
      ANNETY_CRC_STITCH_PIPE=$pipe timeout -k 10 200 python3 bench.py $line --steps 200 --warmup 20 --no-cpu > $O/r${rep}_p${pipe}_$tag.log 2>&1
      echo "rep $rep pipe $pipe $tag $(grep -o '"ms_per_step": [0-9.]*' $O/r${rep}_p${pipe}_$tag.log)"
    done
  done
done
