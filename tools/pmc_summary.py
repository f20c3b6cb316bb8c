#!/usr/bin/env python3
"""Average rocprofv3 --pmc counters per conv kernel instantiation across one or more
run_counter_collection.csv files. usage: python tools/pmc_summary.py dir [dir ...]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "qconv" not in name:
                continue
            m = re.search(r"(qconv\w*)<([^>]*)>", name)
            key = (m.group(1) + "<" + m.group(2).replace(" ", "") + ">") if m else name
            key += " vgpr=%s lds=%s" % (r["VGPR_Count"], r["LDS_Block_Size"])
            vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for key, cs in vals.items():
    print(key)
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    for c in sorted(avg):
        print("   %-28s %16.1f" % (c, avg[c]))
    w = avg.get("SQ_WAVE_CYCLES")
    if w:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if c in avg:
                print("   %-28s %15.1f%%" % (c + "/WAVE_CYCLES", 100 * avg[c] / w))
    print("   median dispatch us (profiled) %.1f" % sorted(dur[key])[len(dur[key]) // 2])
