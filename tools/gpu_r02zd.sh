#!/bin/bash
# per-phase stamps of the current apply (1M fused, 100M multi-pass)
source tools/gpu_lib.sh r02zd
step stamps 300 bash tools/stamps.sh r02zd
