#!/bin/bash
# 16-superstep replays (AGX_MAX_REPLAY=8 = the previous behaviour): parity + headline A/B by knob
source tools/gpu_lib.sh r02zf
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for rep in 1 2; do
  for m in 8 16; do
    AGX_MAX_REPLAY=$m step b20_${m}_$rep 300 python -u bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline --large-actors 0
    AGX_MAX_REPLAY=$m step b200_${m}_$rep 300 python -u bench.py --steps 200 --warmup 16 --no-configs --no-cpu-baseline --large-actors 0
  done
done
