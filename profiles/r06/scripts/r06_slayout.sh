# Linear S layout + short-wave stitch loads: arena parity tests on the product build, then A/B against HEAD's build
# (microbench/libannety_crc_base.so) on frames verify (mixed, chat) and config 3 arena, alternating twice.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-slayout}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_arena.py tests/test_gpu_arena_long.py tests/test_gpu_var_auto.py tests/test_lhc.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
for rep in 1 2; do
  for lib in base new; do
    for line in "--config frames --frames mixed --op verify" "--config frames --frames chat --op verify" "--config 3 --var-path arena"; do
      tag=$(echo "$line" | tr -d ' -' | cut -c1-24)
      if [ $lib = base ]; then L=$GRAFT_REPO_ROOT/microbench/libannety_crc_base.so; else L=$GRAFT_REPO_ROOT/annety_amd/libannety_crc.so; fi
      ANNETY_CRC_LIB=$L timeout -k 10 200 python3 bench.py $line --steps 200 --warmup 20 --no-cpu > $O/r${rep}_${lib}_$tag.log 2>&1
      echo "rep $rep $lib $tag $(grep -o '"ms_per_step": [0-9.]*' $O/r${rep}_${lib}_$tag.log)"
    done
  done
done
