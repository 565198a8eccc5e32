#!/bin/bash
# Round-2 profiles: rocprofv3 kernel stats of the driver's bench command, FETCH/WRITE PMC passes
# (separate runs), then the full driver bench (configs + CPU baseline).
source tools/gpu_lib.sh r02p
step stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02p/stats -o run -- python3 bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r02p/fetch -o run -- python3 bench.py --steps 40 --warmup 4 --no-configs --no-cpu-baseline --large-actors 0
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r02p/write -o run -- python3 bench.py --steps 40 --warmup 4 --no-configs --no-cpu-baseline --large-actors 0
step bench 900 python3 bench.py --steps 20 --warmup 5
