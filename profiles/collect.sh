#!/bin/bash
# Profile the headline bench on a GPU box (run from the repo root via gpurun):
#   1. kernel trace + stats (per-kernel average duration)
#   2. FETCH_SIZE pass, 3. WRITE_SIZE pass (separate --pmc passes, no tracing domains mixed in)
# then summarise into profiles/<tag>_*.  Usage: profiles/collect.sh <tag>
set -e
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
  python3 $R/bench.py --steps 50 --warmup 10 --no-cpu > $OUT/kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex crc32_ --output-format csv -d $OUT/fetch -o run -- \
  python3 $R/bench.py --steps 10 --warmup 2 --prewarm-s 0.3 --no-cpu > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex crc32_ --output-format csv -d $OUT/write -o run -- \
  python3 $R/bench.py --steps 10 --warmup 2 --prewarm-s 0.3 --no-cpu > $OUT/write.log 2>&1
# summaries are written locally after gpurun merges gpurun_out/ back:
#   python3 profiles/parse_prof.py gpurun_out/prof_<tag> <tag>
