#!/bin/bash
source tools/gpu_lib.sh r02h
step delta 600 python -u -m pytest tests/test_gpu_delta_crdt.py tests/test_gpu_typed.py -x -v --timeout 300 --timeout-method thread
step c4d_orset 300 python -u tools/cfg_one.py C4_orset_delta_gossip
step c4d_gc 300 python -u tools/cfg_one.py C4_gcounter_delta_gossip
step ring2048 200 python -u bench.py --steps 200 --warmup 16 --no-configs --large-actors 0 --no-cpu-baseline
AGX_BUCKET_ACTORS=1024 step ring1024 200 python -u bench.py --steps 200 --warmup 16 --no-configs --large-actors 0 --no-cpu-baseline
AGX_BUCKET_ACTORS=512 step ring512 200 python -u bench.py --steps 200 --warmup 16 --no-configs --large-actors 0 --no-cpu-baseline
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
