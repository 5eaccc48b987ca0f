#!/usr/bin/env python3
"""Add C5's per-flush HBM traffic of the radix passes to profiles/pmc_traffic.json (bench.py run_c5's roofline.traffic).

usage: scripts/pmc_c5.py <tag> <c5_batch> <flushes>
Reads gpurun_out/<tag>/c5pmc*/run_counter_collection.csv (one rocprofv3 --pmc pass per counter: FETCH_SIZE and
WRITE_SIZE, in KB; FETCH_SIZE doubled per the gfx950 note of MI355X_MICROARCH.md, as scripts/pmc_summary.py) and
stores the bytes of every rx_scatter dispatch summed over the run, divided by the number of flushes: the traffic of
all radix passes of one flush (the unit bench.py's C5 roofline uses)."""
import csv
import glob
import json
import sys
from collections import defaultdict

tag, batch, flushes = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
tot = defaultdict(float)
for f in sorted(glob.glob("gpurun_out/%s/c5pmc*/run_counter_collection.csv" % tag)):
    for r in csv.DictReader(open(f)):
        if "rx_scatter" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
fetch = tot["FETCH_SIZE"] * 1024 * 2 / flushes
write = tot["WRITE_SIZE"] * 1024 / flushes
path = "profiles/pmc_traffic.json"
d = json.load(open(path))
d.setdefault("c5", {})["rx_scatter"] = {"events_per_launch": batch, "fetch_bytes": fetch, "write_bytes": write,
                                        "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, gpurun_out/%s, per flush "
                                                  "(all radix passes)" % tag}
json.dump(d, open(path, "w"), indent=1)
print("c5 rx_scatter per flush: fetch %.3g B, write %.3g B" % (fetch, write))
