#!/bin/bash
# Round-2 final profiles: rocprofv3 kernel stats of the driver's bench command (headline + 100M),
# FETCH_SIZE / WRITE_SIZE passes over the 1M ring (separate runs), SQ stamps, the full driver bench
source tools/gpu_lib.sh ${R02Y_TAG:-r02y}
step stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R02Y_TAG:-r02y}/stats -o run -- python3 bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${R02Y_TAG:-r02y}/fetch -o run -- python3 bench.py --steps 40 --warmup 4 --no-configs --no-cpu-baseline --large-actors 0
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${R02Y_TAG:-r02y}/write -o run -- python3 bench.py --steps 40 --warmup 4 --no-configs --no-cpu-baseline --large-actors 0
step bench 900 python3 bench.py --steps 20 --warmup 5
step bench200 300 python3 bench.py --steps 200 --warmup 16 --no-configs --no-cpu-baseline --large-actors 0
