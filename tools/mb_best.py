"""Summarize tools/conv_microbench.py output: per shape, the 4 fastest tile configs and the fastest per
kernel family (register-staged < 12 <= LDS-DMA). usage: python tools/mb_best.py mb.log"""
import re
import sys

for line in open(sys.argv[1]):
    if "static" not in line and "dynamic" not in line:
        continue
    r = sorted((float(t), int(c)) for c, t in re.findall(r"cfg(\d+)\s+([\d.]+)us", line))
    fam = {}
    for t, c in r:
        f = "rs" if c < 12 else "glds"
        fam.setdefault(f, (t, c))
    print("%-16s best %s  per family %s" % (line.split()[0], r[:4], fam))
