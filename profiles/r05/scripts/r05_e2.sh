# Encode: partial chunks by lanes 0/1 (tests, probes, bench lines); arena line pass with/without S stores (item 5).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-e2}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_lhc.py tests/test_gpu_fuzz.py -m gpu > $O/pytest.log 2>&1
timeout -k 10 400 python3 microbench/encode_probe.py 0 1 > $O/encode_probe.log 2>&1
for f in mixed chat; do
  timeout -k 10 300 python3 bench.py --config frames --frames $f --op encode --no-cpu > $O/bench_${f}_encode.log 2>&1
done
export SORTED_PROBE_CHILD=1 ANNETY_CRC_LIB=$GRAFT_REPO_ROOT/microbench/libannety_crc_ab.so PROBE_PATH=auto
for b in zipf small; do for lp in 0 1; do
  PROBE_BATCH=$b ANNETY_CRC_LINES_PROBE=$lp timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lines_${b}_$lp -o run -- python3 microbench/sorted_probe.py > $O/lines_${b}_$lp.log 2>&1
done; done
echo done
