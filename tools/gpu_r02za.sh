#!/bin/bash
# branch-free prefetch for the fused variants only: parity + same-box A/B
source tools/gpu_lib.sh r02za
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
AB_REPS=2 PERF_STEPS=40 step ab 600 bash tools/ab.sh r02za akka_amd/lib/ab_prev.so akka_amd/lib/libakka_gpu.so
