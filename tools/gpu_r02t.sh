#!/bin/bash
# inbox loads issued back to back (fast path); ORSet dirty-mask stores: parity + headline + configs
source tools/gpu_lib.sh r02t
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench 300 python -u bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline
step bench200 300 python -u bench.py --steps 200 --warmup 16 --no-configs --no-cpu-baseline --large-actors 0
step c4o 300 python -u tools/cfg_one.py C4_orset_gossip
step c5 300 python -u tools/cfg_one.py C5_power_law_bounded
