#!/bin/bash
# HBM traffic of the bench's kernels at HEAD, one rocprofv3 --pmc pass per counter group (the guide's
# rule: FETCH_SIZE and WRITE_SIZE never share a pass; no tracing domains beside --pmc).
# Usage (GPU box, repo root):  profiles/pmc.sh <tag> <bench args...>
# Writes gpurun_out/pmc_<tag>/{fetch,write,hit}/...; summarise with profiles/pmc.py.
set -e
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
echo "$@" > $OUT/args.txt
cd /tmp && export TMPDIR=/tmp
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  rc=0
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex 'crc32_|lhc_' --output-format csv -d $OUT/p$i -o run -- \
    python3 $R/bench.py --no-cpu --prewarm-s 0.2 --steps 5 --warmup 1 "$@" > $OUT/p$i.log 2>&1 || rc=$?
  echo "pass $i ($P) rc=$rc"
  [ $rc -eq 0 ] || exit $rc  # a failed pass ends the script (set -e would have, without the status)
done
