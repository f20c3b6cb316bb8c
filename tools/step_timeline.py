#!/usr/bin/env python3
"""Per-step timeline of the graph-replayed forward in a rocprofv3 kernel trace of bench.py:
wall time per step, busy (sum of kernel durations), idle gaps and per-kernel-family totals.
A step starts at each smpq::absmax_kernel (the first kernel of the forward).
usage: python tools/step_timeline.py <run_kernel_trace.csv> [nsteps]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
starts = [i for i, r in enumerate(rows) if "absmax_kernel" in r["Kernel_Name"]]
# the timed region's steps: the graph-replayed ones just before the eager roofline region
steps = []
for a, b in zip(starts, starts[1:]):
    steps.append(rows[a:b])
steps = steps[-(nsteps + 5):-5] if len(steps) > nsteps + 5 else steps[:nsteps]
for st in steps:
    t0 = int(st[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in st)
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in st)
    gaps = []
    end = int(st[0]["End_Timestamp"])
    for r in st[1:]:
        s = int(r["Start_Timestamp"])
        if s > end:
            gaps.append((s - end, r["Kernel_Name"][:40]))
        end = max(end, int(r["End_Timestamp"]))
    fam = collections.Counter()
    for r in st:
        k = r["Kernel_Name"].split("<")[0].split("(")[0].replace("void ", "")
        fam[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print("step: %d kernels, wall %.1f us, busy %.1f us, gaps %.1f us (%d gaps; largest %s)" % (
        len(st), (t1 - t0) / 1e3, busy / 1e3, sum(g for g, _ in gaps) / 1e3, len(gaps),
        ", ".join("%.1f before %s" % (g / 1e3, n) for g, n in sorted(gaps, reverse=True)[:3])))
print("kernel families (last step, us):", {k: round(v, 1) for k, v in fam.most_common()})
