#!/bin/bash
source tools/gpu_lib.sh r02d
step diag16 120 python -u tools/replay_diag.py
AGX_MAX_REPLAY=8 step diag8 120 python -u tools/replay_diag.py
