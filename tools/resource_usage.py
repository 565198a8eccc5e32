#!/usr/bin/env python3
"""Summarise hipcc `-Rpass-analysis=kernel-resource-usage` remarks: one line per kernel
(demangled name, VGPRs, AGPRs, spills, scratch bytes/lane, dynamic stack, LDS, occupancy).

  hipcc ... -c --cuda-device-only -Rpass-analysis=kernel-resource-usage x.hip 2> ru.txt
  python tools/resource_usage.py ru.txt [name-filter]
"""
import re
import subprocess
import sys


def parse(path):
    kernels, cur = [], None
    for line in open(path, errors="replace"):
        m = re.search(r"remark: (.*?) \[-Rpass-analysis", line)
        if not m:
            continue
        body = m.group(1).strip()
        if body.startswith("Function Name:"):
            cur = {"name": body.split(":", 1)[1].strip()}
            kernels.append(cur)
        elif cur is not None and ":" in body:
            k, v = body.split(":", 1)
            cur[k.strip()] = v.strip()
    return kernels


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
        return out[:len(names)]
    except OSError:
        return names


def main():
    ks = parse(sys.argv[1])
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    names = demangle([k["name"] for k in ks])
    for k, n in zip(ks, names):
        if flt and flt not in n:
            continue
        print(f"{n[:110]:110s} vgpr={k.get('VGPRs', '?'):>4} agpr={k.get('AGPRs', '?'):>3} "
              f"spill={k.get('VGPRs Spill', '?'):>3} scratch={k.get('ScratchSize [bytes/lane]', '?'):>4} "
              f"dynstack={k.get('Dynamic Stack', '?'):>5} lds={k.get('LDS Size [bytes/block]', '?'):>6} "
              f"occ={k.get('Occupancy [waves/SIMD]', '?')}")


if __name__ == "__main__":
    main()
