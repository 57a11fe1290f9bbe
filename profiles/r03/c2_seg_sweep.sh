set -e
O=$GRAFT_REPO_ROOT/gpurun_out/c2seg
mkdir -p $O
for rep in 1 2; do
for seg in 65536 4096 8192 16384 32768; do
  ANNETY_CRC_SEG=$seg timeout -k 10 100 python bench.py --config 2 --steps 20 --warmup 3 --no-cpu > $O/c2_seg${seg}_$rep.log 2>&1
done
done
