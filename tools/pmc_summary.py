"""Summarise rocprofv3 counter CSVs (tools/f2_pmc.sh): per kernel symbol, the median of each
counter over its dispatches.   python tools/pmc_summary.py gpurun_out/f2pmc"""
import collections
import csv
import glob
import os
import statistics
import sys

d = sys.argv[1]
per = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        per[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in per.items():
    print(k)
    for c in sorted(cs):
        print(f"   {c:28s} {statistics.median(cs[c]):16.0f}")
