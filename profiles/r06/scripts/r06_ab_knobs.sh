# A/B of A/B-build knob settings (microbench/libannety_crc_ab.so through ANNETY_CRC_LIB) on bench lines, alternating
# twice; every bench line checks its results against the oracle before timing.
# Usage: r06_ab_knobs.sh <out> "<lines>" "<name>:<VAR=V[,VAR=V]>" ...   (lines: c3a c3s fmv fcv)
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/$1; shift; mkdir -p $O; cd $GRAFT_REPO_ROOT
LINES=$1; shift
export TMPDIR=/tmp ANNETY_CRC_LIB=$GRAFT_REPO_ROOT/microbench/libannety_crc_ab.so
args() {
  case $1 in
    c3a) echo "--config 3 --var-path arena";; c3s) echo "--config 3 --var-path sorted";;
    fmv) echo "--config frames --frames mixed --op verify";; fcv) echo "--config frames --frames chat --op verify";;
    fme) echo "--config frames --frames mixed --op encode";; fce) echo "--config frames --frames chat --op encode";;
  esac
}
for rep in 1 2; do
  for S in "$@"; do
    name=${S%%:*}; envs=${S#*:}
    for line in $LINES; do
      rc=0
      env $(echo $envs | tr ',' ' ') timeout -k 10 200 python3 bench.py $(args $line) --steps 200 --warmup 20 --no-cpu > $O/r${rep}_${name}_$line.log 2>&1 || rc=$?
      echo "rep $rep $name $line rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/r${rep}_${name}_$line.log)"
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
