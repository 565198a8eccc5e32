#!/bin/bash
# final tree: full GPU suite, smoke, driver bench
source tools/gpu_lib.sh r02zn
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 900 python3 bench.py --steps 20 --warmup 5
