#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc runs: mean counter value per dispatch for each kernel (gpurun_out/<tag>/pmc*/)."""
import csv
import glob
import sys
from collections import defaultdict

tag = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else ""
acc = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob("gpurun_out/%s/pmc*/run_counter_collection.csv" % tag)):
    per = defaultdict(float)
    meta = {}
    for r in csv.DictReader(open(f)):
        if kern not in r["Kernel_Name"]:
            continue
        key = (r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1], r["Dispatch_Id"], r["Counter_Name"])
        per[key] += float(r["Counter_Value"])
    for (k, d, c), v in per.items():
        acc[k][c].append(v)
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print("   %-24s %14.4g  (n=%d)" % (c, sum(v) / len(v), len(v)))
