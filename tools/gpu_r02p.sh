#!/bin/bash
# per-kernel times of C5 with the skew pre-pass (rocprofv3 kernel trace)
source tools/gpu_lib.sh r02p
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step c5prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02p/prof -o c5 -- python3 -u tools/cfg_one.py C5_power_law_bounded
