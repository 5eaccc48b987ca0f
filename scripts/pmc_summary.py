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

# --traffic: write profiles/pmc_traffic.json (HBM bytes per launch per kernel) for bench.py's roofline.traffic.
# FETCH_SIZE / WRITE_SIZE are in KB; FETCH_SIZE is doubled per the gfx950 note of MI355X_MICROARCH.md (it tallies
# 128-B memory-side read requests at 64 B).
if len(sys.argv) > 3 and sys.argv[3] == "--traffic":
    import json
    events = int(sys.argv[4])
    launches = int(sys.argv[5]) if len(sys.argv) > 5 else 1  # matcher launches per step (fused sub-batches)
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, gpurun_out/%s" % tag, "events_per_launch": events,
           "launches_per_step": launches,
           "note": "events_per_launch: the bench step's events; bytes are per launch (a step runs launches_per_step)",
           "kernels": {}}
    for k, cs in acc.items():
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            f = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024 * 2
            w = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024
            out["kernels"][k.split("<")[0]] = {"fetch_bytes": f, "write_bytes": w}
    json.dump(out, open("profiles/pmc_traffic.json", "w"), indent=1)
    print("wrote profiles/pmc_traffic.json")
