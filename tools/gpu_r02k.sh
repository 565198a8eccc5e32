#!/bin/bash
source tools/gpu_lib.sh r02k
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for c in C4_orset_gossip C4_gcounter_gossip C4_orset_delta_gossip C4_gcounter_delta_gossip; do
  step $c 300 python -u tools/cfg_one.py $c
done
