# Kernel times of the linear S layout against HEAD's build: rocprofv3 kernel trace of config 3 arena and frames
# verify (mixed) with each library.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-slkt}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for lib in base new; do
  if [ $lib = base ]; then L=$GRAFT_REPO_ROOT/microbench/libannety_crc_base.so; else L=$GRAFT_REPO_ROOT/annety_amd/libannety_crc.so; fi
  for cfg in c3 fmv; do
    if [ $cfg = c3 ]; then A="--config 3 --var-path arena"; else A="--config frames --frames mixed --op verify"; fi
    ANNETY_CRC_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${lib}_$cfg -o run -- python3 bench.py $A --steps 200 --warmup 20 --no-cpu > $O/${lib}_$cfg.log 2>&1
    python3 profiles/r06/kt_summary.py $O/${lib}_$cfg $O/kt_${lib}_$cfg.csv
    echo "== $lib $cfg"; cat $O/kt_${lib}_$cfg.csv | grep -E "lines|stitch"
  done
done
