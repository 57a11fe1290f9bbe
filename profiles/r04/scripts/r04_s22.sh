# Round-4 pass at HEAD: full GPU suite, smoke, the driver's bench command plain and under the kernel tracer,
# and the other configs' bench lines (config 3 automatic and sorted, config 2) under the kernel tracer.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s22}; mkdir -p $O; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_driver -o kt -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/kt_driver_bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c3 -o kt -- python3 bench.py --config 3 > $O/kt_c3_bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c3s -o kt -- python3 bench.py --config 3 --var-path sorted > $O/kt_c3s_bench.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c2 -o kt -- python3 bench.py --config 2 > $O/kt_c2_bench.log 2>&1
rm -f $O/kt_*/kt_kernel_trace.csv
echo done
