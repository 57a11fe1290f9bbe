set -e
O=gpurun_out/s5c
mkdir -p $O
timeout -k 10 120 python -u -m pytest tests/test_gpu_arena_streams.py -x -v --timeout 100 --timeout-method thread > $O/pytest_streams.log 2>&1
timeout -k 10 60 ./microbench/stitch_mb > $O/stitch_mb.log 2>&1
for i in 1 2; do
  ANNETY_CRC_ARENA_EVENTS=1 timeout -k 10 120 python bench.py --config 3 --steps 200 --warmup 10 --no-cpu --sample-check > $O/c3_events_$i.log 2>&1
  timeout -k 10 120 python bench.py --config 3 --steps 200 --warmup 10 --no-cpu --sample-check > $O/c3_slots_$i.log 2>&1
done
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo done
