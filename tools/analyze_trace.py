#!/usr/bin/env python3
"""Per-layer breakdown of a rocprofv3 kernel trace of bench.py (R50, one forward = 48 qconv launches).

usage: python tools/analyze_trace.py gpurun_out/prof/run_kernel_trace.csv [batch]
Prints, for the last forward in the trace: each quantized conv's time, algorithmic TOP/s, the
MFMA floor (limbs x alg ops at 5 POPS) and the HBM floor (int8-limb input + fp32 output (+fp32
residual) at 8 TB/s), and a per-kernel-name total per forward.
"""
import collections
import csv
import sys

path = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
L = int(sys.argv[3]) if len(sys.argv) > 3 else 2
rows = list(csv.DictReader(open(path)))
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
q = [r for r in rows if "qconv_" in r["Kernel_Name"]]
nfwd = len(q) // 48
shapes = []
H, inp = 56, 64
for li, (nb, planes) in enumerate(zip([3, 4, 6, 3], [64, 128, 256, 512])):
    for b in range(nb):
        s = 2 if (li > 0 and b == 0) else 1
        Ho = H // s
        shapes += [(inp, planes, 1, 1, H, H, 0), (planes, planes, 3, s, H, Ho, 0), (planes, planes * 4, 1, 1, Ho, Ho, 1)]
        inp, H = planes * 4, Ho
tot = troof = 0
print(" cin  cout k s  Hin      us  TOP/s  mfma_us  hbm_us")
for (cin, cout, k, s, H, Ho, res), r in zip(shapes, q[-48:]):
    d = dur(r)
    ops = 2 * B * Ho * Ho * cout * cin * k * k
    mf = L * ops / 5e15 * 1e6
    hb = (B * H * H * cin * L + B * Ho * Ho * cout * 4 * (2 if res else 1)) / 8e12 * 1e6
    tot += d
    troof += max(mf, hb)
    print(f"{cin:4d} {cout:5d} {k} {s} {H:4d} {d:8.1f} {ops / d / 1e6:6.1f} {mf:7.1f} {hb:7.1f}")
print(f"qconv total {tot:.0f} us/forward, per-layer roofline {troof:.0f} us ({troof / tot:.1%})")
# all kernels, per forward (the trace holds warmup + timed forwards)
agg = collections.defaultdict(float)
for r in rows:
    agg[r["Kernel_Name"][:70]] += dur(r)
print("\nper-forward totals (us), %d forwards in trace:" % nfwd)
for k, v in sorted(agg.items(), key=lambda kv: -kv[1])[:16]:
    print(f"{v / nfwd:9.1f}  {k}")
