#!/bin/bash
# graph upload at capture; headline at the driver's step count; per-phase stamps; C4 ORSet traffic
source tools/gpu_lib.sh r02r
step bench 300 python -u bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline --large-actors 0
step bench2 300 python -u bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline --large-actors 0
step stamps 300 bash tools/stamps.sh r02r
step orset_fetch 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r02r/of -o of -- python3 -u tools/cfg_one.py C4_orset_gossip
step orset_write 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r02r/ow -o ow -- python3 -u tools/cfg_one.py C4_orset_gossip
