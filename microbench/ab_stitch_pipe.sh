set -e
O=gpurun_out/s5g
mkdir -p $O
for i in 1 2 3; do
  ANNETY_CRC_STITCH_PIPE=0 timeout -k 10 120 python bench.py --config 3 --steps 300 --warmup 10 --no-cpu --sample-check > $O/c3_pipe0_$i.log 2>&1
  ANNETY_CRC_STITCH_PIPE=1 timeout -k 10 120 python bench.py --config 3 --steps 300 --warmup 10 --no-cpu --sample-check > $O/c3_pipe1_$i.log 2>&1
done
ANNETY_CRC_STITCH_PIPE=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_arena_streams.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "arena or config3 or zipf or var or stream" > $O/pytest_pipe1.log 2>&1
echo done
