#!/bin/bash
# Whole-payload vs segment+combine path on long-payload shapes (bench.py, device-resident, no CPU leg),
# then the segment size on the split path.
set -e
cd "$(dirname "$0")/.."
run() { timeout -k 10 120 python bench.py --config 2 --payloads $1 --len $2 --steps 30 --warmup 5 --no-cpu --prewarm-s 0.5; }
for shape in "4096 4194304" "1024 1048576" "16 67108864" "1 1073741824" "1 268435456"; do
  set -- $shape
  for seg in 32768 65536 131072; do
    echo "== n=$1 len=$2 split=1 seg=$seg"
    ANNETY_CRC_SPLIT=1 ANNETY_CRC_SEG=$seg run $1 $2
  done
done
