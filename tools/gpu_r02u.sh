#!/bin/bash
# DPP wave scans + two-barrier block scans: full GPU parity, A/B vs the previous commit, driver bench
source tools/gpu_lib.sh r02u
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
AB_REPS=2 PERF_STEPS=40 step ab 600 bash tools/ab.sh r02u akka_amd/lib/ab_prev.so akka_amd/lib/libakka_gpu.so
step bench 600 python -u bench.py --steps 20 --warmup 5
