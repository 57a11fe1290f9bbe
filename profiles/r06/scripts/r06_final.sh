# Round-6 final pass at HEAD (after the PMC summaries of r06_measure.sh are committed under profiles/r06/pmc): the
# whole GPU suite, smoke(), the driver's default bench command and every other bench line (their traffic now read
# from the committed summaries).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-final}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py > $O/bench_c1.log 2>&1
for L in "c2:--config 2" "c3a:--config 3" "c3s:--config 3 --var-path sorted" "c4:--config 4" \
         "fmv:--config frames --frames mixed --op verify" "fcv:--config frames --frames chat --op verify" \
         "fme:--config frames --frames mixed --op encode" "fce:--config frames --frames chat --op encode"; do
  T=${L%%:*}; A=${L#*:}
  timeout -k 10 300 python3 bench.py $A --no-cpu > $O/bench_$T.log 2>&1
done
python3 - $O <<'PY'
import json, glob, sys, os
for f in sorted(glob.glob(sys.argv[1] + "/bench_*.log")):
    for line in open(f):
        if line.startswith("{"):
            j = json.loads(line); r = j["roofline"]
            print(os.path.basename(f), j["value"], j["ms_per_step"], r["frac"], r.get("traffic"), (r.get("traffic_refused") or {}).get("why"))
PY
echo done
