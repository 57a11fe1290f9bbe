set -e
O=$GRAFT_REPO_ROOT/gpurun_out/s2; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_stream -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config 3 --var-path stream --steps 50 --warmup 5 --no-cpu --sample-check > $O/kt_stream.log 2>&1
cd $GRAFT_REPO_ROOT
bash profiles/r04/scripts/r04_scale_inputs.sh r04_scale
