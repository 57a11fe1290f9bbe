# Counting sort grid: payloads per thread 1 / 2 / 4 / 8 (ANNETY_CRC_BUCKET_PER, A/B build), config 3 sorted path.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s12}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 0 1; do for p in 1 2 4 8; do
  ANNETY_CRC_BUCKET_PER=$p timeout -k 10 200 python3 microbench/sorted_probe.py 0 > $O/per${p}_$rep.log 2>&1
done; done
ANNETY_CRC_BUCKET_PER=4 PROBE_BATCH=small timeout -k 10 200 python3 microbench/sorted_probe.py 0 > $O/small_per4.log 2>&1
PROBE_BATCH=small timeout -k 10 200 python3 microbench/sorted_probe.py 0 > $O/small_per1.log 2>&1
echo done
