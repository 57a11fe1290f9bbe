set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04b; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_arena.py tests/test_gpu_fuzz.py tests/test_gpu_var_auto.py tests/test_gpu_nt.py tests/test_gpu_fullsize.py::test_config3_full_bitexact -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_arena.log 2>&1
profiles/ab_run.sh r04b/ab_c3 ab/libannety_crc_4205b95.so 3 --config 3 --steps 200 --warmup 20 --no-cpu --sample-check > $O/ab_c3.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config 3 --steps 100 --warmup 10 --no-cpu --sample-check > $O/kt_c3.log 2>&1
cd $GRAFT_REPO_ROOT
bash profiles/r04/scripts/r04_scale_inputs.sh r04_scale
