#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV outputs: mean counter value per dispatch, per kernel."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for pat in sys.argv[1:]:
    for f in sorted(glob.glob(pat)):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(agg.items()):
    if "agx" not in k:
        continue
    waves = d.get("SQ_WAVES")
    wv = sum(waves) / len(waves) if waves else None
    print(k)
    for c, v in sorted(d.items()):
        m = sum(v) / len(v)
        extra = f"  per-wave={m / wv:10.1f}" if wv and c.startswith("SQ_") and c != "SQ_WAVES" else ""
        print(f"   {c:26s} mean/dispatch={m:14.1f}{extra}")
