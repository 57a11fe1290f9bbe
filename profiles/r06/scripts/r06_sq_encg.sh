# SQ counters of the fused encode with 4 and with 8 lanes per frame (ANNETY_CRC_ENC_G through the A/B library),
# on the mixed and chat frames lines; one rocprofv3 --pmc pass per counter group, no trace domains.
# Usage: r06_sq_encg.sh <out>
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp ANNETY_CRC_LIB=$R/microbench/libannety_crc_ab.so
for G in 4 8; do
  for F in mixed chat; do
    i=0
    for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" \
             "SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVES SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC"; do
      i=$((i+1)); rc=0
      ANNETY_CRC_ENC_G=$G timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex 'lhc_' --output-format csv \
        -d $O/g${G}_$F/p$i -o run -- python3 $R/bench.py --no-cpu --prewarm-s 0.2 --steps 5 --warmup 1 \
        --config frames --frames $F --op encode > $O/g${G}_${F}_p$i.log 2>&1 || rc=$?
      echo "G $G $F pass $i rc=$rc"
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections, os
o = sys.argv[1]
for d in sorted(glob.glob(o + "/g*_*")):
    if not os.path.isdir(d): continue
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(d + "/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        print(os.path.basename(d), k, {c: round(sum(v) / len(v), 1) for c, v in sorted(cs.items())})
PY
