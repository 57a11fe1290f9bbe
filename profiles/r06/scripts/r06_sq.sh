# SQ / TA / TCP counters of the frames-verify line (lines + stitch), one rocprofv3 --pmc pass per group, no trace
# domains beside --pmc (the guide's rule). Usage: r06_sq.sh <out> [bench args...]
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/$1; shift; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVES SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC" \
         "TA_BUSY_avr TA_BUSY_max TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1)); rc=0
  timeout -s KILL 60 rocprofv3 --pmc $P --kernel-include-regex 'crc32_|lhc_' --output-format csv -d $O/p$i -o run -- \
    python3 $R/bench.py --no-cpu --prewarm-s 0.2 --steps 5 --warmup 1 "$@" > $O/p$i.log 2>&1 || rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(o + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("annety_crc::(anonymous namespace)::", "").split("(")[0]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k, {c: round(sum(v) / len(v), 1) for c, v in sorted(cs.items())})
PY
