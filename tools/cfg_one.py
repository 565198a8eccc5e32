#!/usr/bin/env python3
"""Time one BASELINE config of bench.py (the same workload / warmup / timed supersteps).

    python tools/cfg_one.py C4_orset_gossip [--quick]"""
import json
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import bench  # noqa: E402


def main():
    name = sys.argv[1]
    quick = "--quick" in sys.argv
    cfgs = bench.other_configs(quick, only=name)
    print(json.dumps({name: cfgs[name]}))


if __name__ == "__main__":
    main()
