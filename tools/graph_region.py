#!/usr/bin/env python3
"""The graph-replayed timed region of bench.py in a rocprofv3 kernel trace, per layer.

usage: python tools/graph_region.py <run_kernel_trace.csv> [launches_per_slice steps rsteps slices]

bench.py's tail in the trace (round 5): [timed: steps graph replays, each `slices` batch slices
of `launches_per_slice` quantized convs on their own queues] [whole-batch eager region: 1 + rsteps
steps] [roofline region: 1 + rsteps steps of the same slices, one launch at a time]. A slice is a
dependency chain (its kernels never overlap each other); the chains run concurrently, one per
hardware queue (Queue_Id). For each layer: the mean duration in the graph region (concurrent with
the other slice), the duration of the same layer launched alone in the roofline region, and the
step's wall time vs the summed kernel time per chain. NB: rocprofv3's per-dispatch overhead
delays the second slice's start in a traced replay (~2 ms); tools/timeline_probe.py measures the
timeline without a profiler.
"""
import collections
import csv
import sys


def dur(r):
    return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3


def short(name):
    n = name.replace("void ", "").replace("smpq::", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:60]


def main():
    path = sys.argv[1]
    per = int(sys.argv[2]) if len(sys.argv) > 2 else 53
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    rsteps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    slices = int(sys.argv[5]) if len(sys.argv) > 5 else 2
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    q = [r for r in rows if "qconv" in r["Kernel_Name"]]
    eager_n = (rsteps + 1) * per + (rsteps + 1) * per * slices
    roof = q[-rsteps * per * slices:]
    timed = q[-eager_n - steps * per * slices:-eager_n]
    if len(timed) != steps * per * slices:
        raise SystemExit("trace too short for %d steps" % steps)
    lay = collections.defaultdict(list)
    walls, busy = [], []
    for s in range(steps):
        st = timed[s * per * slices:(s + 1) * per * slices]
        chains = collections.defaultdict(list)
        for r in st:
            chains[r["Queue_Id"]].append(r)
        if len(chains) != slices or any(len(c) != per for c in chains.values()):
            raise SystemExit("step %d: chains by queue %s" % (s, {k: len(v) for k, v in chains.items()}))
        t0 = min(int(r["Start_Timestamp"]) for r in st)
        t1 = max(int(r["End_Timestamp"]) for r in st)
        walls.append((t1 - t0) / 1e3)
        busy.append(sum(dur(r) for r in st) / slices)
        for c in chains.values():
            for i, r in enumerate(c):
                lay[i].append((dur(r), short(r["Kernel_Name"]), r["Grid_Size_X"], r["Workgroup_Size_X"]))
    rl = collections.defaultdict(list)
    for k in range(rsteps * slices):
        for i, r in enumerate(roof[k * per:(k + 1) * per]):
            rl[i].append(dur(r))
    print("%3s %9s %9s %6s  %-60s %9s %5s" % ("#", "graph_us", "eager_us", "ratio", "kernel (graph slice)", "grid", "wg"))
    tg = te = 0.0
    for i in range(per):
        d = [x[0] for x in lay[i]]
        g = sum(d) / len(d)
        e = sum(rl[i]) / len(rl[i])
        tg += g
        te += e
        _, name, grid, wg = lay[i][0]
        print("%3d %9.1f %9.1f %6.2f  %-60s %9s %5s" % (i, g, e, g / e, name, grid, wg))
    w = sorted(walls)[len(walls) // 2]
    b = sorted(busy)[len(busy) // 2]
    print("graph region: median step wall %.1f us (qconv span), qconv time per slice chain %.1f us "
          "(sum over the %d chains %.1f us, concurrency %.2f)" % (w, b, slices, b * slices, b * slices / w))
    print("per slice: sum of graph-region layer means %.1f us; roofline region (the same slice launched alone) %.1f us"
          % (tg, te))


if __name__ == "__main__":
    main()
