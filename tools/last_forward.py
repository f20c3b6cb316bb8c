#!/usr/bin/env python3
"""Per-kernel and per-conv times of the LAST ResNet-50 forward in a rocprofv3 kernel trace.
usage: python tools/last_forward.py <run_kernel_trace.csv> [batch]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
q = [i for i, r in enumerate(rows) if "qconv" in r["Kernel_Name"]]
last = q[-53:]
st = last[0]
while st > 0 and "image_quantize" not in rows[st]["Kernel_Name"]:
    st -= 1
seg = rows[max(st - 1, 0):last[-1] + 4]
agg, cnt = collections.defaultdict(float), collections.Counter()
for r in seg:
    k = r["Kernel_Name"].split("(")[0][:70]
    agg[k] += dur(r)
    cnt[k] += 1
for k, v in sorted(agg.items(), key=lambda kv: -kv[1]):
    print(f"{v:9.1f} us {cnt[k]:4d}x  {k}")
print("forward total %.1f us" % sum(agg.values()))
shapes = [("stem", 3, 64, 7, 2, 224, 112)]
H, inp = 56, 64
for li, (nb, planes) in enumerate(zip([3, 4, 6, 3], [64, 128, 256, 512])):
    for b in range(nb):
        s = 2 if (li > 0 and b == 0) else 1
        Ho = H // s
        if b == 0:
            shapes.append(("ds", inp, planes * 4, 1, s, H, Ho))
        shapes += [("c1", inp, planes, 1, 1, H, H), ("c2", planes, planes, 3, s, H, Ho), ("c3", planes, planes * 4, 1, 1, Ho, Ho)]
        inp, H = planes * 4, Ho
tot = collections.defaultdict(float)
for sh, i in zip(shapes, last):
    r = rows[i]
    d = dur(r)
    n, cin, cout, k, s, H, Ho = sh
    ops = 2 * B * Ho * Ho * cout * cin * k * k
    tot[n] += d
    print(f"{n:4s} {cin:5d} {cout:5d} {k} {s} {H:4d} {d:8.1f}us {ops / d / 1e6:7.1f}TOP/s  {r['Kernel_Name'].split('(')[0][20:]}")
print({k: round(v, 1) for k, v in tot.items()})
