set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fz
L=gpurun_out/fz/probe.log
: > $L
for r in 1 2; do
  ANNETY_CRC_ARENA_FUSED=0 timeout -k 10 120 python microbench/fused_probe.py >> $L 2>&1 || exit 1
  for v in 0 1 2 3 4 8 11; do
    ANNETY_CRC_FUSED_VAR=$v timeout -k 10 120 python microbench/fused_probe.py >> $L 2>&1 || exit 1
  done
done
cat $L
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/fz/prof_fused -o run -- python3 $GRAFT_REPO_ROOT/microbench/fused_probe.py 50 > $GRAFT_REPO_ROOT/gpurun_out/fz/prof_fused.log 2>&1 || exit 2
