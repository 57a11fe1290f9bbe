# Re-measure bench lines at HEAD: for each line named on the command line, the PMC passes (profiles/pmc.sh ->
# pmc.py summary stamped with the source digests), a rocprofv3 kernel trace of the bench command, and the bench line.
# Usage: bash profiles/r06/scripts/r06_measure.sh <outdir> <line>...   lines: c1 c2 c3a c3s c4 fmv fcv fme fce
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/$1; shift; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
args_of() {
  case $1 in
    c1) echo "" ;; c2) echo "--config 2" ;; c3a) echo "--config 3" ;; c3s) echo "--config 3 --var-path sorted" ;;
    c4) echo "--config 4" ;;
    fmv) echo "--config frames --frames mixed --op verify" ;; fcv) echo "--config frames --frames chat --op verify" ;;
    fme) echo "--config frames --frames mixed --op encode" ;; fce) echo "--config frames --frames chat --op encode" ;;
  esac
}
for L in "$@"; do
  if [ "$L" = "e1" ] || [ "$L" = "e3" ]; then  # the host-memory (PCIe) paths of configs 1 and 3
    C=${L#e}
    timeout -k 10 600 python3 bench.py --config $C --e2e --no-cpu --steps 50 > $O/bench_e2e_c$C.log 2>&1
    tail -c 600 $O/bench_e2e_c$C.log
    continue
  fi
  A=$(args_of $L)
  echo "== $L: $A"
  if [ "$L" != "c4" ]; then
    bash profiles/pmc.sh m_$L $A --sample-check > $O/pmc_$L.log 2>&1
    python3 profiles/pmc.py gpurun_out/pmc_m_$L $O/pmc_$L.json > /dev/null
    find gpurun_out/pmc_m_$L -name "*counter_collection.csv" -delete
  fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$L -o run -- \
     python3 $GRAFT_REPO_ROOT/bench.py $A --no-cpu --sample-check --steps 100 > $O/kt_$L.log 2>&1)
  find $O/kt_$L -name "*kernel_trace.csv" -delete
  if [ "$L" = "c1" ]; then
    timeout -k 10 300 python3 bench.py > $O/bench_$L.log 2>&1
  else
    timeout -k 10 300 python3 bench.py $A --no-cpu > $O/bench_$L.log 2>&1
  fi
  tail -c 400 $O/bench_$L.log
done
echo done
