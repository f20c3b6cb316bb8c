#!/usr/bin/env python3
"""Join tools/pmc_layers.sh's two PMC passes to bench.py's layer table: per quantized-conv launch of
the eager roofline region (the last N x 3 dispatches, N = the launches of a step: 53 for R50), the instruction mix per wave (VALU, SALU,
LDS, VMEM) against its MFMA cycles, and the wave states. Diagnostics only.

usage: python tools/pmc_layers.py <outdir>"""
import csv
import glob
import os
import re
import sys

O = sys.argv[1]
N, R = 53, 3


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    rows = {}
    for r in csv.DictReader(open(f)):
        if "qconv" not in r["Kernel_Name"]:
            continue
        k = int(r["Dispatch_Id"])
        rows.setdefault(k, {"name": r["Kernel_Name"], "vgpr": r["VGPR_Count"], "agpr": r["Accum_VGPR_Count"]})
        rows[k][r["Counter_Name"]] = rows[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [rows[k] for k in sorted(rows)][-N * R:]


layers = []
log = open(os.path.join(O, "p1.log")).read().splitlines()
try:
    i = next(j for j, l in enumerate(log) if l.startswith("launch"))
    # the layer table's rows (one per launch of a step) end at its "total" line: N of any config
    N = next(j for j, l in enumerate(log[i + 1:]) if l.startswith("total"))
    layers = [l[:33] + l[33:43] for l in log[i + 1:i + 1 + N]]
except StopIteration:
    layers = [""] * N
p1, p2 = load(os.path.join(O, "p1")), load(os.path.join(O, "p2"))
groups = {}
print("%-43s %5s %7s %6s %6s %6s %6s %5s %5s %5s %5s %6s" % (
    "launch (t_us)", "vgpr", "waves", "VALU/w", "SALU/w", "LDS/w", "MFMAc/w", "V/MF", "wait", "istl", "actv", "mfma%"))
for j in range(N):
    a = [p1[r * N + j] for r in range(R)]
    b = [p2[r * N + j] for r in range(R)]
    def m(lst, k):
        return sum(x.get(k, 0.0) for x in lst) / len(lst)
    w = m(a, "SQ_WAVES")
    mf = m(a, "SQ_VALU_MFMA_BUSY_CYCLES")
    wc = m(b, "SQ_WAIT_ANY") + m(b, "SQ_WAIT_INST_ANY") + m(b, "SQ_ACTIVE_INST_ANY")
    gui = m(b, "GRBM_GUI_ACTIVE")
    print("%-43s %5s %7d %6.0f %6.0f %6.0f %6.0f %5.2f %5.2f %5.2f %5.2f %6.1f" % (
        layers[j] if j < len(layers) else "", a[0]["vgpr"], w, m(a, "SQ_INSTS_VALU") / w, m(a, "SQ_INSTS_SALU") / w,
        m(a, "SQ_INSTS_LDS") / w, mf / w, m(a, "SQ_INSTS_VALU") / max(mf / 16, 1),
        m(b, "SQ_WAIT_ANY") / wc, m(b, "SQ_WAIT_INST_ANY") / wc, m(b, "SQ_ACTIVE_INST_ANY") / wc,
        100 * mf / max(gui * 128, 1)))
    # per conv group: time-weighted MFMA busy, VALU and SALU per MFMA, wave-state shares
    lab = layers[j] if j < len(layers) else ""
    mm = re.match(r"\s*(\d+)->\s*(\d+) k(\d)\s+(\d+)->\s*(\d+)\s+\S+\s+([\d.]+)", lab)
    if not mm:
        continue
    k, h, ho, t = int(mm.group(3)), int(mm.group(4)), int(mm.group(5)), float(mm.group(6))
    g = ("stem+pool" if k == 7 else "3x3 stride 2" if (k == 3 and ho < h) else "3x3 %d^2" % ho if k == 3
         else "downsample 1x1/s2" if ho < h else "1x1 %d^2" % ho)
    acc = groups.setdefault(g, [0.0] * 7)
    nmf = max(mf / 16, 1)
    for q, v in enumerate((t, t * mf / max(gui * 128, 1), t * m(a, "SQ_INSTS_VALU") / nmf,
                           t * m(a, "SQ_INSTS_SALU") / nmf, t * m(b, "SQ_WAIT_ANY") / wc,
                           t * m(b, "SQ_WAIT_INST_ANY") / wc, 1.0)):
        acc[q] += v
print()
print("%-20s %9s %8s %9s %9s %8s %8s %4s" % ("group", "t_us", "mfma%", "VALU/MF", "SALU/MF", "wait%", "istall%", "n"))
for g, (t, mfp, va, sa, wt, ist, n) in sorted(groups.items(), key=lambda kv: -kv[1][0]):
    print("%-20s %9.1f %8.1f %9.2f %9.2f %8.1f %8.1f %4d" % (g, t, 100 * mfp / t, va / t, sa / t, 100 * wt / t,
                                                           100 * ist / t, n))
