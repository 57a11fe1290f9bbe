# Same-box A/B of two full library builds (ANNETY_CRC_LIB): bench lines alternating twice, then a rocprofv3 kernel
# trace of each line with each library. Usage: r06_ab_libs.sh <out> <libA> <libB> <lines...> (c3a c3s fmv fcv fme fce)
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
LA=$2; LB=$3; shift 3
args() {
  case $1 in
    c3a) echo "--config 3 --var-path arena";;
    c3s) echo "--config 3 --var-path sorted";;
    fmv) echo "--config frames --frames mixed --op verify";;
    fcv) echo "--config frames --frames chat --op verify";;
    fme) echo "--config frames --frames mixed --op encode";;
    fce) echo "--config frames --frames chat --op encode";;
  esac
}
for rep in 1 2; do
  for lib in A B; do
    if [ $lib = A ]; then L=$LA; else L=$LB; fi
    for line in "$@"; do
      ANNETY_CRC_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python3 bench.py $(args $line) --steps 200 --warmup 20 --no-cpu > $O/r${rep}_${lib}_$line.log 2>&1
      echo "rep $rep $lib $line $(grep -o '"ms_per_step": [0-9.]*' $O/r${rep}_${lib}_$line.log)"
    done
  done
done
for lib in A B; do
  if [ $lib = A ]; then L=$LA; else L=$LB; fi
  for line in "$@"; do
    ANNETY_CRC_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${lib}_$line -o run -- python3 bench.py $(args $line) --steps 200 --warmup 20 --no-cpu > $O/kt_${lib}_$line.log 2>&1
    python3 profiles/r06/kt_summary.py $O/kt_${lib}_$line $O/kt_${lib}_$line.csv > /dev/null
    echo "== $lib $line"; grep -E "lines|stitch|sorted|extent|place" $O/kt_${lib}_$line.csv
  done
done
