#!/usr/bin/env python3
"""Summarize a rocprofv3 --kernel-trace --stats run of bench.py: per-kernel totals and the
average duration of the quantized-conv launches (to check bench.py's event-timed avg_launch_ms).
usage: python tools/rocprof_summary.py <run_kernel_stats.csv> [run_kernel_trace.csv [L steps rsteps]]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("%-90s %8s %12s %10s %6s" % ("kernel", "calls", "total_ms", "avg_us", "pct"))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print("%-90s %8s %12.3f %10.2f %6.2f" % (r["Name"][:90], r["Calls"], float(r["TotalDurationNs"]) / 1e6,
                                              float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
q = [r for r in rows if "qconv" in r["Name"]]
calls = sum(int(r["Calls"]) for r in q)
qt = sum(float(r["TotalDurationNs"]) for r in q)
print("quantized conv (qconv*): %d launches, total %.3f ms, avg %.5f ms/launch, %.1f%% of GPU time"
      % (calls, qt / 1e6, qt / max(calls, 1) / 1e6, 100 * qt / tot))

if len(sys.argv) > 2:
    # bench.py's regions at the end of the trace: [timed: steps x L graph-replayed] [1 untimed eager
    # step] [roofline: rsteps x L eager, event-timed]
    L = int(sys.argv[3]) if len(sys.argv) > 3 else 53
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    rsteps = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    tr = [r for r in csv.DictReader(open(sys.argv[2])) if "qconv" in r["Kernel_Name"]]
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in tr]
    roof = dur[-rsteps * L:]
    print("roofline region (last %d launches, eager, one launch at a time): avg %.5f ms/launch, %.3f ms/step"
          % (len(roof), sum(roof) / len(roof), sum(roof) / rsteps))
