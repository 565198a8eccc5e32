#!/bin/bash
# ORSet runs element-batch-outer: CRDT parity, C4 ORSet rate and traffic, headline
source tools/gpu_lib.sh r02s
step par 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_benched.py tests/test_gpu_delta_crdt.py -x -q --timeout 300 --timeout-method thread -k "crdt or orset or ORSet or C4 or gossip"
step c4o 300 python -u tools/cfg_one.py C4_orset_gossip
step orset_fetch 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r02s/of -o of -- python3 -u tools/cfg_one.py C4_orset_gossip
step orset_write 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r02s/ow -o ow -- python3 -u tools/cfg_one.py C4_orset_gossip
step bench 300 python -u bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline --large-actors 0
